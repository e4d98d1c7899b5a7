"""GPU placement services behind the partner stages.

The reference shells out for each of these searches:

- `bwa mem -M` of the one-end-anchored pairs vs the genome (Anchored_Fusion.py:188) and of the
  anchored split reads (functions.py:716): `Reference` + `af_place`, the K2 seed-and-extend in
  placement mode (every region scoring >= T per query), rendered by bwa_records with bwa's
  record rules;
- BLAT of tails and candidates vs the genome, the candidate blocks and the anchor
  (functions.py:341, 530, 966, 1007, 1071, 1122, 1244): `Placer`, the `place(targets, queries,
  preset)` callback of partner.py, runs the BLAT restatement (blat.py, csrc/blat.hip) with each
  call's options and returns PSL lines.

`Reference` joins contigs with runs of 512 N and indexes them once; seeds cannot cross an N run
and extension cannot score across one.  Parity with bwa / BLAT themselves is unpinned: neither
is available (SURVEY.md §8 c).  The kernels are bit-exact against oracle/af_oracle.c `afo_place`
and oracle/blat.c `afo_blat` (tests/test_gpu_place.py, tests/test_gpu_blat.py).
"""
import bisect
import ctypes
import re

import numpy as np

from . import _lib

SEP = 512  # N run between contigs
WINDOW = 300  # long-query window (step WINDOW // 2)
HIT_DTYPE = np.dtype([("query", "<i4"), ("flag", "<i4"), ("score", "<i4"), ("q_start", "<i4"), ("q_end", "<i4"),
                      ("q_size", "<i4"), ("matches", "<i4"), ("n_cigar", "<i4"), ("t_start", "<i8"),
                      ("t_end", "<i8"), ("cigar", "<u4", (32,))])
assert HIT_DTYPE.itemsize == 176

# the genome bwa calls (AF:188, fn:716): bwa mem defaults (-k 19 -T 30)
PRESET_PARAMS = {
    "genome_bwa": (30, 0),
}

_OPS = "MIDNSHP=X"


def cigar_string(ops):
    return "".join(f"{int(c) >> 4}{_OPS[int(c) & 15]}" for c in ops)


def pack_queries(seqs):
    stride = max(1, max((len(s) for s in seqs), default=1))
    if stride > _lib.AF_MAX_READ:
        raise ValueError(f"query longer than {_lib.AF_MAX_READ}")
    buf = np.full((len(seqs), stride), ord("N"), dtype=np.uint8)
    lens = np.zeros(len(seqs), dtype=np.int32)
    for i, s in enumerate(seqs):
        b = s.encode() if isinstance(s, str) else bytes(s)
        buf[i, :len(b)] = np.frombuffer(b, dtype=np.uint8)
        lens[i] = len(b)
    return buf, lens


def concat_contigs(contigs):
    """Contigs [(name, seq)] -> (joined bytes, contig offsets); SEP N's between contigs."""
    parts, offsets, off = [], [], 0
    for k, (_, seq) in enumerate(contigs):
        if k:
            parts.append("N" * SEP)
            off += SEP
        offsets.append(off)
        parts.append(seq)
        off += len(seq)
    blob = "".join(parts).encode()
    return (blob if blob else b"N"), offsets


GENOME_INDEX_MIN = 1 << 25  # references from 32 Mbp up get the GPU-built genome index


def index_kind(total):
    """"hash" (host-built 16-mer hash of both strands, af_index_build) or "genome" (GPU-built
    direct table, af_index_build_genome) for a reference of `total` bases; AF_INDEX_KIND=hash|genome
    forces one."""
    import os
    k = os.environ.get("AF_INDEX_KIND", "auto")
    if k in ("hash", "genome"):
        return k
    return "genome" if total >= GENOME_INDEX_MIN else "hash"


class Reference:
    """Contigs [(name, seq)] indexed on the GPU for af_place."""

    def __init__(self, contigs, device=0, ctx=None):
        self.names = [n for n, _ in contigs]
        self.lens = [len(s) for _, s in contigs]
        blob, self.offsets = concat_contigs(contigs)
        self.total = len(blob)
        L = _lib.lib()
        self._own_ctx = ctx is None
        if ctx is None:
            ctx = ctypes.c_void_p()
            _lib.check(None, L.af_ctx_create(int(device), ctypes.byref(ctx)), "af_ctx_create")
        self.ctx = ctx
        self.idx = ctypes.c_void_p()
        self.kind = index_kind(len(blob))
        build = L.af_index_build_genome if self.kind == "genome" else L.af_index_build
        _lib.check(self.ctx, build(self.ctx, blob, len(blob), ctypes.byref(self.idx)),
                   "af_index_build_genome" if self.kind == "genome" else "af_index_build")

    @classmethod
    def from_device(cls, blob_t, names, lens, offsets, device=0, ctx=None):
        """A genome already joined in HBM (torch uint8 tensor laid out as concat_contigs does: contigs
        at `offsets`, SEP N's between them) indexed by af_index_build_genome_device."""
        self = cls.__new__(cls)
        self.names, self.lens, self.offsets = list(names), [int(v) for v in lens], [int(v) for v in offsets]
        self.total = int(blob_t.numel())
        if self.total < 1 or not blob_t.is_cuda or not blob_t.is_contiguous():
            raise ValueError("blob_t must be a non-empty contiguous device tensor")
        if self.offsets[-1] + self.lens[-1] > self.total:
            raise ValueError("contigs extend past the blob")
        L = _lib.lib()
        self._own_ctx = ctx is None
        if ctx is None:
            ctx = ctypes.c_void_p()
            _lib.check(None, L.af_ctx_create(int(device), ctypes.byref(ctx)), "af_ctx_create")
        self.ctx = ctx
        self.idx = ctypes.c_void_p()
        self.kind = "genome"
        _lib.check(self.ctx, L.af_index_build_genome_device(self.ctx, blob_t.data_ptr(), self.total,
                                                             ctypes.byref(self.idx)), "af_index_build_genome_device")
        return self

    def close(self):
        L = _lib.lib()
        if getattr(self, "idx", None):
            L.af_index_free(self.idx)
            self.idx = None
        if getattr(self, "_own_ctx", False) and getattr(self, "ctx", None):
            L.af_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def raw_hits(self, seqs, params=None, max_hits=16):
        """af_place on packed queries -> (hits structured array [n, max_hits], n_hits [n])."""
        buf, lens = pack_queries(seqs)
        n = len(seqs)
        hits = np.zeros((n, max_hits), dtype=HIT_DTYPE)
        nh = np.zeros(n, dtype=np.int32)
        if n == 0:
            return hits, nh
        p = params or _lib.default_params()
        rc = _lib.lib().af_place(self.ctx, self.idx, buf.ctypes.data, n, buf.shape[1], lens.ctypes.data,
                                 ctypes.byref(p), max_hits, hits.ctypes.data, nh.ctypes.data)
        _lib.check(self.ctx, rc, "af_place")
        return hits, nh

    def place_device(self, queries_t, n_queries_t, stride, hits_t, n_hits_t, lens_t=None, params=None,
                     max_hits=16, stream=None, ctx=None):
        """af_place_device: queries_t uint8 [cap, stride] on the device, n_queries_t an int32
        device scalar (clamped to cap), hits_t a device buffer of cap * max_hits * 176 bytes
        (view it on the host with HIT_DTYPE), n_hits_t int32 [cap].  Asynchronous on stream.
        ctx: the context whose queue heads and traceback scratch the launch uses (default this
        Reference's).  A context's placement must be stream-ordered with every other K2 or
        placement enqueued on that context (they share its scratch): placements running
        concurrently on several streams need a context of their own each, and an AlignerGroup
        slot's ``aligner.ctx`` may only be used on that slot's own stream."""
        from .align import _stream_handle
        cap = int(queries_t.shape[0])
        if queries_t.dim() != 2 or int(queries_t.shape[1]) < int(stride):
            raise ValueError("queries_t must be [cap, >= stride]")
        if lens_t is not None and lens_t.numel() < cap:
            raise ValueError("lens_t holds fewer than cap entries")
        if hits_t.numel() * hits_t.element_size() < cap * max_hits * HIT_DTYPE.itemsize:
            raise ValueError("hits_t holds fewer than cap * max_hits hits")
        if n_hits_t.numel() < cap:
            raise ValueError("n_hits_t holds fewer than cap entries")
        p = params or _lib.default_params()
        c = self.ctx if ctx is None else ctx
        _lib.check(c, _lib.lib().af_place_device(
            c, self.idx, queries_t.data_ptr(), n_queries_t.data_ptr(), cap, int(stride),
            None if lens_t is None else lens_t.data_ptr(), ctypes.byref(p), int(max_hits), hits_t.data_ptr(),
            n_hits_t.data_ptr(), _stream_handle(stream)), "af_place_device")

    def locate(self, t_start, t_end):
        """Concatenated forward coordinates -> (contig index, local start, local end) or None."""
        k = bisect.bisect_right(self.offsets, int(t_start)) - 1
        if k < 0:
            return None
        s, e = int(t_start) - self.offsets[k], int(t_end) - self.offsets[k]
        if s < 0 or e > self.lens[k] or e <= s:
            return None
        return k, s, e


def preset_params(preset="genome_bwa"):
    """af_params of the genome bwa calls: bwa mem's defaults (-k 19 -T 30)."""
    T, _ = PRESET_PARAMS[preset]
    p = _lib.default_params()
    p.T = T
    p.min_seed_len = 19
    return p


class Placer:
    """The `place(targets, queries, preset)` callback of partner.py (BLAT with the preset's
    options, blat.PRESETS) and the genome `Reference` of the bwa calls.

    Targets are indexed once per distinct target set (and tile step)."""

    def __init__(self, device=0, max_hits=16, reference_factory=None, tile_factory=None):
        from . import blat
        self.device, self.max_hits = device, max_hits
        self.factory = reference_factory or (lambda contigs: Reference(contigs, device=device))
        self.tile_factory = tile_factory or (lambda contigs, step: blat.TileReference(contigs, step, device=device))
        self._refs, self._tiles = {}, {}

    @staticmethod
    def _key(targets):
        return tuple((n, hash(s)) for n, s in targets)

    def reference(self, targets):
        key = self._key(targets)
        ref = self._refs.get(key)
        if ref is None:
            ref = self.factory([(n, s) for n, s in targets])
            self._refs[key] = ref
        return ref

    def tiles(self, targets, step):
        key = (self._key(targets), int(step))
        ref = self._tiles.get(key)
        if ref is None:
            ref = self.tile_factory([(n, s) for n, s in targets], int(step))
            self._tiles[key] = ref
        return ref

    def params(self, preset):
        return preset_params(preset)

    def __call__(self, targets, queries, preset):
        from . import blat
        header = ["psLayout version 3\n", "\n"]
        if not targets or not queries:
            return header
        p = blat.params(preset)
        ref = self.tiles(targets, p.step_size)
        # queries longer than the kernel's read limit (the anchor transcript itself, fn:341/966)
        # are searched as overlapping windows; rows keep the full query's name, size and coordinates
        pieces = []  # (name, window seq, offset, full length)
        for name, seq in queries:
            if len(seq) <= _lib.AF_MAX_READ:
                pieces.append((name, seq, 0, len(seq)))
            else:
                for off in range(0, max(1, len(seq) - WINDOW // 2), WINDOW // 2):
                    pieces.append((name, seq[off:off + WINDOW], off, len(seq)))
        rows, nr = ref.search([w for _, w, _, _ in pieces], p, blat.MAX_ROWS)
        return header + blat.psl_lines(ref, [(nm, w) for nm, w, _, _ in pieces], rows, nr,
                                       offsets=[o for _, _, o, _ in pieces], full_sizes=[f for _, _, _, f in pieces])

    def close(self):
        for r in list(self._refs.values()) + list(self._tiles.values()):
            r.close()
        self._refs.clear()
        self._tiles.clear()


_FASTA_NAME = re.compile(r"^>(\S+)")
