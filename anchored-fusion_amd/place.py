"""The BLAT searches behind the partner stages.

The reference shells out to BLAT for the tails and candidates vs the genome, the candidate
blocks and the anchor (functions.py:341, 530, 966, 1007, 1071, 1122, 1244).  `Placer` is the
`place(targets, queries, preset)` callback of partner.py: it runs the BLAT restatement (blat.py,
csrc/blat.hip) with each call's options and returns PSL lines.  Targets are joined with runs of
512 N (`concat_contigs`); a tile cannot cross an N run.  Parity with BLAT itself is unpinned
(absent, SURVEY.md §8 c); the kernel is bit-exact against oracle/blat.c `afo_blat`
(tests/test_gpu_blat.py).  The genome `bwa mem` calls (S4 / S5) are genome.py.
"""
import numpy as np

from . import _lib

SEP = 512  # N run between contigs


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


class Placer:
    """The `place(targets, queries, preset)` callback of partner.py (BLAT with the preset's
    options, blat.PRESETS).  Targets are indexed once per distinct target set and tile step."""

    def __init__(self, device=0, tile_factory=None):
        from . import blat
        self.device = device
        self.on_device = tile_factory is None   # TileReference (GPU) searches; tests inject the oracle
        self.tile_factory = tile_factory or (lambda contigs, step: blat.TileReference(contigs, step, device=device))
        self._tiles = {}

    @staticmethod
    def _key(targets):
        return tuple((n, hash(s)) for n, s in targets)

    def tiles(self, targets, step):
        key = (self._key(targets), int(step))
        ref = self._tiles.get(key)
        if ref is None:
            ref = self.tile_factory([(n, s) for n, s in targets], int(step))
            self._tiles[key] = ref
        return ref

    def __call__(self, targets, queries, preset):
        from . import blat
        header = ["psLayout version 3\n", "\n"]
        if not targets or not queries:
            return header
        p = blat.params(preset)
        ref = self.tiles(targets, p.step_size)
        lines = [[] for _ in queries]
        short = [i for i, (_, sq) in enumerate(queries) if len(sq) <= _lib.AF_MAX_READ]
        if short:  # every row of each query (the rows past MAX_ROWS from the search's spill pool)
            rows, nr, extra = ref.search_all([queries[i][1] for i in short], p)
            for k, i in enumerate(short):
                lines[i] = blat.psl_lines(ref, [queries[i]], rows[k:k + 1], nr[k:k + 1],
                                          extra={0: extra[k]} if k in extra else None)
        # a query longer than a read (the anchor transcript itself, fn:341 / fn:966) is searched
        # whole, as BLAT takes it (af_blat_long)
        for i, (nm, sq) in enumerate(queries):
            if len(sq) > _lib.AF_MAX_READ:
                rows, n_all, blocks, off = ref.search_long(sq, p)
                if n_all > len(rows):  # more rows than the first call returned: all of them
                    rows, n_all, blocks, off = ref.search_long(sq, p, max_rows=n_all)
                lines[i] = blat.psl_lines_long(ref, nm, sq, rows, blocks, off)
        out = list(header)
        for ln in lines:
            out += ln
        return out

    def close(self):
        for r in self._tiles.values():
            r.close()
        self._tiles.clear()

