"""The BLAT searches of the partner stages on the GPU (af_tile_index_build / af_blat, csrc/blat.hip).

The reference shells out to BLAT at functions.py:341 (homologs), 530 (split-read tails), 966
(anchor vs candidate blocks), 1007/1071 (partner halves vs candidate blocks), 1122 (anchored
halves vs the anchor) and 1244 (candidate validation vs the genome), each with its own options.
`PRESETS` carries those options; `TileReference` is a target indexed for one step size;
`psl_lines` renders the rows in BLAT's PSL column layout (psLayout version 3), which the
consumers read (partner.py, blocks.py).  The search itself is restated (include/afgpu.h,
af_blat_params), bit-exact vs oracle/blat.c; parity with the BLAT binary is
unpinned.
"""
import ctypes

import numpy as np

from . import _lib
from .place import concat_contigs, pack_queries

PSL_DTYPE = np.dtype([(n, "<i4") for n in (
    "query", "strand", "score", "matches", "mismatches", "n_count", "q_num_insert", "q_base_insert", "t_num_insert",
    "t_base_insert", "q_start", "q_end", "q_size", "block_count")] + [
    ("t_start", "<i8"), ("t_end", "<i8"), ("block_sizes", "<i4", (16,)), ("q_starts", "<i4", (16,)),
    ("t_starts", "<i8", (16,))])
assert PSL_DTYPE.itemsize == 328
BLOCK_DTYPE = np.dtype([("size", "<i4"), ("q_start", "<i4"), ("t_start", "<i8")])  # af_psl_block
TILE = 11
MAX_ROWS = 16
LONG_MAX = 131072   # AF_BLAT_LONG_MAX: the longest query af_blat_long searches whole
LONG_ROWS = 4096    # rows a long search returns (every row is counted)
CAP_NAMES = ("hits", "clumps", "parts", "rows")  # af_blat_caps' counters, in order

# the reference's option sets (functions.py call sites); rep_match None = BLAT's default
PRESETS = {
    "homologs": dict(step_size=3, rep_match=10000, min_score=50, min_identity=80),          # fn:341
    "split_tail": dict(min_score=20),                                                        # fn:530
    "candidate_homolog": dict(step_size=3, min_score=20, min_match=2, min_identity=0),      # fn:966
    "anchored_split": dict(step_size=3, min_score=12, min_match=2, min_identity=90),        # fn:1007/1071/1122
    "genome_validate": dict(step_size=3, min_score=20, min_match=3, min_identity=90),       # fn:1244
}


class BlatParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("step_size", "min_match", "rep_match", "min_score", "min_identity",
                                                "max_gap", "max_intron")]


def params(preset=None, **kw):
    """af_blat_params: BLAT's defaults, the preset's options, then kw.  Without an explicit
    -repMatch, BLAT's default of 1024 (11-mer tiles) scales with tileSize / stepSize."""
    p = BlatParams()
    _lib.lib().af_blat_params_default(ctypes.byref(p))
    opts = dict(PRESETS[preset]) if preset else {}
    opts.update(kw)
    for k, v in opts.items():
        setattr(p, k, v)
    if "rep_match" not in opts:
        p.rep_match = 1024 * TILE // p.step_size
    return p


class TileReference:
    """Contigs [(name, seq)] (or a joined device blob, from_device) as a BLAT target with one
    tile step."""

    def __init__(self, contigs, step_size=TILE, device=0, ctx=None):
        self.names = [n for n, _ in contigs]
        self.lens = [len(s) for _, s in contigs]
        blob, self.offsets = concat_contigs(contigs)
        self.total = len(blob)
        self.step = int(step_size)
        self._open(device, ctx)
        _lib.check(self.ctx, _lib.lib().af_tile_index_build(self.ctx, blob, len(blob), self.step, ctypes.byref(self.idx)),
                   "af_tile_index_build")

    def _open(self, device, ctx):
        self.device = int(device)
        self._own_ctx = ctx is None
        if ctx is None:
            ctx = ctypes.c_void_p()
            _lib.check(None, _lib.lib().af_ctx_create(int(device), ctypes.byref(ctx)), "af_ctx_create")
        self.ctx = ctx
        self.idx = ctypes.c_void_p()

    @classmethod
    def from_device(cls, blob_t, names, lens, offsets, step_size=TILE, device=0, ctx=None):
        self = cls.__new__(cls)
        self.names, self.lens, self.offsets = list(names), [int(v) for v in lens], [int(v) for v in offsets]
        self.total = int(blob_t.numel())
        self.step = int(step_size)
        if not blob_t.is_cuda or not blob_t.is_contiguous():
            raise ValueError("blob_t must be a contiguous device tensor")
        self._open(device, ctx)
        _lib.check(self.ctx, _lib.lib().af_tile_index_build_device(self.ctx, blob_t.data_ptr(), self.total, self.step,
                                                                    ctypes.byref(self.idx)),
                   "af_tile_index_build_device")
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

    def search(self, seqs, p, max_rows=MAX_ROWS):
        """af_blat -> (rows [n, max_rows] PSL_DTYPE, n_rows [n])."""
        buf, lens = pack_queries(seqs)
        n = len(seqs)
        rows = np.zeros((n, max_rows), dtype=PSL_DTYPE)
        nr = np.zeros(n, dtype=np.int32)
        if n:
            _lib.check(self.ctx, _lib.lib().af_blat(self.ctx, self.idx, buf.ctypes.data, n, buf.shape[1],
                                                   lens.ctypes.data, ctypes.byref(p), max_rows, rows.ctypes.data,
                                                   nr.ctypes.data), "af_blat")
        return rows, nr

    def search_all(self, seqs, p, spill_cap=None):
        """Every row of every query, as BLAT prints them: (rows [n, MAX_ROWS], n_rows [n], {query:
        [its rows past MAX_ROWS]}) -- af_blat_device with the spill pool on this reference's
        context (device buffers made here; the rows come back to the host)."""
        import torch
        n = len(seqs)
        if not n:
            return np.zeros((0, MAX_ROWS), PSL_DTYPE), np.zeros(0, np.int32), {}
        buf, lens = pack_queries(seqs)
        dev = torch.device("cuda", self.device)
        q_t = torch.from_numpy(buf).to(dev)
        l_t = torch.from_numpy(lens).to(dev)
        n_t = torch.tensor([n], dtype=torch.int32, device=dev)
        rows_t = torch.zeros(n * MAX_ROWS * PSL_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        nr_t = torch.zeros(n, dtype=torch.int32, device=dev)
        cap = spill_cap or max(1024, 4 * n)
        sp = dict(rows=torch.zeros(cap * PSL_DTYPE.itemsize, dtype=torch.uint8, device=dev),
                  q=torch.zeros(cap, dtype=torch.int32, device=dev), n=torch.zeros(1, dtype=torch.int32, device=dev))
        stream = torch.cuda.current_stream(dev)
        self.spill_to(sp["rows"], sp["q"], sp["n"])
        try:
            self.search_device(q_t, n_t, buf.shape[1], rows_t, nr_t, lens_t=l_t, p=p, stream=stream)
        finally:
            self.spill_to()
        torch.cuda.synchronize(dev)
        ns = int(sp["n"].item())
        if ns > cap:
            raise _lib.AFError(f"af_blat spill pool of {cap} rows overflowed ({ns} rows)")
        rows = rows_t.cpu().numpy().view(PSL_DTYPE).reshape(n, MAX_ROWS)
        extra = spilled_rows(sp["rows"][:ns * PSL_DTYPE.itemsize].cpu().numpy().view(PSL_DTYPE),
                             sp["q"][:ns].cpu().numpy())
        return rows, nr_t.cpu().numpy(), extra

    def search_long(self, seq, p, max_rows=LONG_ROWS):
        """af_blat_long: one query longer than a read (the anchor transcript, fn:341 / fn:966) searched
        whole -> (rows [k] PSL_DTYPE best first, n_rows (all rows), blocks BLOCK_DTYPE, block_off
        [k + 1]): row i's blocks are blocks[block_off[i]:block_off[i + 1]]."""
        b = seq.encode() if isinstance(seq, str) else bytes(seq)
        if len(b) > LONG_MAX:
            raise ValueError(f"query longer than {LONG_MAX}")
        rows = np.zeros(max_rows, dtype=PSL_DTYPE)
        nr = np.zeros(1, np.int32)
        off = np.zeros(max_rows + 1, np.int64)
        nb = np.zeros(1, np.int64)
        cap = 1 << 16
        while True:
            blocks = np.zeros(cap, dtype=BLOCK_DTYPE)
            rc = _lib.lib().af_blat_long(self.ctx, self.idx, b, len(b), ctypes.byref(p), int(max_rows), rows.ctypes.data,
                                         nr.ctypes.data, blocks.ctypes.data, cap, off.ctypes.data, nb.ctypes.data)
            if rc == _lib.AF_E_CAPACITY and int(nb[0]) > cap:
                cap = int(nb[0])
                continue
            _lib.check(self.ctx, rc, "af_blat_long")
            k = min(int(nr[0]), int(max_rows))
            return rows[:k].copy(), int(nr[0]), blocks[:int(off[k])].copy(), off[:k + 1].copy()

    def search_device(self, queries_t, n_queries_t, stride, rows_t, n_rows_t, lens_t=None, p=None, max_rows=MAX_ROWS,
                      stream=None, first_t=None):
        """af_blat_device on device buffers (rows_t: cap * max_rows * 328 bytes); first_t (an int32
        device word, optional): search only the queries from *first_t on (af_blat_device_range)."""
        from .align import _stream_handle
        cap = self._check_device(queries_t, stride, rows_t, n_rows_t, lens_t, max_rows)
        _lib.check(self.ctx, _lib.lib().af_blat_device_range(
            self.ctx, self.idx, queries_t.data_ptr(), None if first_t is None else first_t.data_ptr(),
            n_queries_t.data_ptr(), cap, int(stride), None if lens_t is None else lens_t.data_ptr(),
            ctypes.byref(p or params()), int(max_rows), rows_t.data_ptr(), n_rows_t.data_ptr(),
            _stream_handle(stream)), "af_blat_device_range")

    def search_device_begin(self, queries_t, n_queries_t, stride, rows_t, n_rows_t, lens_t=None, p=None,
                            max_rows=MAX_ROWS, stream=None):
        """af_blat_device_begin: the per-strand pass of a device search (the heavy strands' clumps
        left as jobs); search_device_end finishes it for the live queries."""
        from .align import _stream_handle
        cap = self._check_device(queries_t, stride, rows_t, n_rows_t, lens_t, max_rows)
        _lib.check(self.ctx, _lib.lib().af_blat_device_begin(
            self.ctx, self.idx, queries_t.data_ptr(), n_queries_t.data_ptr(), cap, int(stride),
            None if lens_t is None else lens_t.data_ptr(), ctypes.byref(p or params()), int(max_rows),
            rows_t.data_ptr(), n_rows_t.data_ptr(), _stream_handle(stream)), "af_blat_device_begin")

    def search_device_end(self, live_t=None, stream=None):
        """af_blat_device_end: the deferred strands and the rows of the queries with live_t[q] != 0
        (uint8 device flags; None: every query)."""
        from .align import _stream_handle
        _lib.check(self.ctx, _lib.lib().af_blat_device_end(
            self.ctx, None if live_t is None else live_t.data_ptr(), _stream_handle(stream)), "af_blat_device_end")

    @staticmethod
    def _check_device(queries_t, stride, rows_t, n_rows_t, lens_t, max_rows):
        cap = int(queries_t.shape[0])
        if queries_t.dim() != 2 or int(queries_t.shape[1]) < int(stride):
            raise ValueError("queries_t must be [cap, >= stride]")
        if rows_t.numel() * rows_t.element_size() < cap * max_rows * PSL_DTYPE.itemsize or n_rows_t.numel() < cap:
            raise ValueError("rows_t / n_rows_t too small for cap queries")
        if lens_t is not None and lens_t.numel() < cap:
            raise ValueError("lens_t holds fewer than cap entries")
        return cap

    def spill_to(self, rows_t=None, query_t=None, n_t=None):
        """af_blat_spill: later device searches on this reference's context append each query's
        rows past max_rows to rows_t (uint8 [cap * 328]) with their query index in query_t, the
        count in n_t (int32 device word the caller zeroes); no arguments: unregister."""
        if rows_t is None:
            _lib.check(self.ctx, _lib.lib().af_blat_spill(self.ctx, None, None, None, 0), "af_blat_spill")
            return
        cap = min(rows_t.numel() * rows_t.element_size() // PSL_DTYPE.itemsize, int(query_t.numel()))
        _lib.check(self.ctx, _lib.lib().af_blat_spill(self.ctx, rows_t.data_ptr(), query_t.data_ptr(), n_t.data_ptr(),
                                                      int(cap)), "af_blat_spill")

    def query_caps_to(self, counts_t=None, cap=0):
        """af_blat_query_caps: later device searches on this reference's context count their cap
        events per query in counts_t (int32 [4 * cap], zeroed by the caller: counter k of query q
        at k * cap + q); no arguments: unregister."""
        if counts_t is None:
            _lib.check(self.ctx, _lib.lib().af_blat_query_caps(self.ctx, None, 0), "af_blat_query_caps")
            return
        if counts_t.numel() < len(CAP_NAMES) * int(cap):
            raise ValueError("counts_t holds fewer than 4 * cap counters")
        _lib.check(self.ctx, _lib.lib().af_blat_query_caps(self.ctx, counts_t.data_ptr(), int(cap)),
                   "af_blat_query_caps")

    def heavy_stats(self):
        """af_blat_heavy_stats of the last device search: strands deferred, their jobs, jobs aligned,
        strands chained (synchronises)."""
        out = np.zeros(4, np.int32)
        _lib.check(self.ctx, _lib.lib().af_blat_heavy_stats(self.ctx, out.ctypes.data), "af_blat_heavy_stats")
        return dict(zip(("deferred", "jobs", "aligned", "chained"), (int(v) for v in out)))

    def caps(self, reset=True):
        """af_blat_caps: query strands / queries at each of the search's caps since the last reset
        (synchronises)."""
        out = np.zeros(len(CAP_NAMES), np.int32)
        _lib.check(self.ctx, _lib.lib().af_blat_caps(self.ctx, out.ctypes.data, int(bool(reset))), "af_blat_caps")
        return dict(zip(CAP_NAMES, (int(v) for v in out)))

    def locate(self, t_start, t_end):
        import bisect
        k = bisect.bisect_right(self.offsets, int(t_start)) - 1
        if k < 0:
            return None
        s, e = int(t_start) - self.offsets[k], int(t_end) - self.offsets[k]
        if s < 0 or e > self.lens[k] or e <= s:
            return None
        return k, s, e


PSL_ORDER = ("score", "strand", "t_start", "q_start", "t_end", "q_end")  # psl_before: score desc, then ascending


def spilled_rows(rows, query):
    """The spill pool's rows (PSL_DTYPE [n], query index [n]) grouped per query in the search's row
    order (score desc, strand, tStart, qStart, tEnd, qEnd; rows equal on all six -- the pool holds
    them in atomic order -- by their bytes, so the order does not depend on the run): {query: [row,
    ...]}.  They follow the query's kept rows."""
    out = {}
    if len(rows) == 0:
        return out
    order = np.lexsort((rows["q_end"], rows["t_end"], rows["q_start"], rows["t_start"], rows["strand"],
                        -rows["score"].astype(np.int64), query))
    for i in order:
        out.setdefault(int(query[i]), []).append(rows[i])
    for q, rs in out.items():  # exact ties of the six keys: by the row's bytes
        keys = [tuple(int(r[f]) for f in PSL_ORDER) for r in rs]
        if len(set(keys)) < len(keys):
            out[q] = [r for _, _, r in sorted(((-k[0],) + k[1:], r.tobytes(), r) for k, r in zip(keys, rs))]
    return out


def psl_lines_long(ref, name, seq, rows, blocks, block_off):
    """PSL lines of one long query's rows (search_long): every block of each row."""
    out = []
    L = len(seq)
    for i, r in enumerate(rows):
        loc = ref.locate(r["t_start"], r["t_end"])
        if loc is None:
            continue
        tk, ts, te = loc
        base = ref.offsets[tk]
        bl = blocks[int(block_off[i]):int(block_off[i + 1])]
        qs = [int(b["q_start"]) for b in bl]  # '-': on the reverse-complemented query, as BLAT prints them
        f = [int(r["matches"]), int(r["mismatches"]), 0, int(r["n_count"]), int(r["q_num_insert"]),
             int(r["q_base_insert"]), int(r["t_num_insert"]), int(r["t_base_insert"]), "-" if r["strand"] else "+", name,
             L, int(r["q_start"]), int(r["q_end"]), ref.names[tk], ref.lens[tk], ts, te, len(bl),
             ",".join(str(int(b["size"])) for b in bl) + ",", ",".join(map(str, qs)) + ",",
             ",".join(str(int(b["t_start"]) - base) for b in bl) + ","]
        out.append("\t".join(map(str, f)) + "\n")
    return out


def psl_lines(ref, queries, rows, nr, offsets=None, full_sizes=None, extra=None):
    """PSL lines (21 columns, psLayout 3) of the rows of queries [(name, seq)].  offsets /
    full_sizes: a query that is a window of a longer sequence reports the full query's size and
    coordinates (offset added; '-' strand blocks mapped on the full reverse complement).  extra:
    {query index: [rows past the kept ones]} (spilled_rows), printed after them."""
    out = []
    for i, (name, seq) in enumerate(queries):
        off = 0 if offsets is None else int(offsets[i])
        full = len(seq) if full_sizes is None else int(full_sizes[i])
        mine = [rows[i, k] for k in range(max(int(nr[i]), 0))] + (extra.get(i, []) if extra else [])
        for r in mine:
            loc = ref.locate(r["t_start"], r["t_end"])
            if loc is None:
                continue
            tk, ts, te = loc
            base = ref.offsets[tk]
            nb = int(r["block_count"])
            strand = "-" if r["strand"] else "+"
            if r["strand"]:  # rc-window coordinates -> rc-full coordinates
                qs = [full - (off + len(seq)) + int(v) for v in r["q_starts"][:nb]]
            else:
                qs = [off + int(v) for v in r["q_starts"][:nb]]
            f = [int(r["matches"]), int(r["mismatches"]), 0, int(r["n_count"]), int(r["q_num_insert"]),
                 int(r["q_base_insert"]), int(r["t_num_insert"]), int(r["t_base_insert"]), strand, name, full,
                 off + int(r["q_start"]), off + int(r["q_end"]), ref.names[tk], ref.lens[tk], ts, te, nb,
                 ",".join(str(int(v)) for v in r["block_sizes"][:nb]) + ",", ",".join(map(str, qs)) + ",",
                 ",".join(str(int(v) - base) for v in r["t_starts"][:nb]) + ","]
            out.append("\t".join(map(str, f)) + "\n")
    return out
