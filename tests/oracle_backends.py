"""CPU oracle stand-ins for the GPU search services -- TEST INFRASTRUCTURE ONLY.

They let the end-to-end pipeline (anchored_fusion_amd.pipeline) run on CPU in the
`-m "not gpu"` suite. The product never imports this module.
"""
import bisect

import numpy as np

import afpkg  # noqa: F401
import oracle
from anchored_fusion_amd.align import AlignResult
from anchored_fusion_amd.place import concat_contigs, pack_queries


class OracleTileReference:
    """The BLAT restatement's CPU contract (oracle/blat.c) behind Placer's tile_factory."""

    def __init__(self, contigs, step):
        self.names = [n for n, _ in contigs]
        self.lens = [len(s) for _, s in contigs]
        blob, self.offsets = concat_contigs(contigs)
        self.total = len(blob)
        self.step = int(step)
        self.tiles = oracle.OracleTiles(blob, self.step)

    def search(self, seqs, p, max_rows=16):
        buf, lens = pack_queries(seqs)
        op = oracle.blat_params(**{f: getattr(p, f) for f, _ in p._fields_})
        return self.tiles.blat(buf, lens, op, max_rows, threads=8)

    def search_all(self, seqs, p, all_rows=256):
        """TileReference.search_all's contract on the oracle: the first MAX_ROWS rows per query and
        the rest (up to all_rows) as {query: [rows]}."""
        from anchored_fusion_amd.blat import MAX_ROWS
        rows, nr = self.search(seqs, p, all_rows)
        extra = {k: list(rows[k, MAX_ROWS:int(c)]) for k, c in enumerate(nr) if c > MAX_ROWS}
        return rows[:, :MAX_ROWS].copy(), np.minimum(nr, MAX_ROWS).astype(np.int32), extra

    def search_long(self, seq, p, max_rows=4096):
        """TileReference.search_long's contract on the oracle (afo_blat_long)."""
        op = oracle.blat_params(**{f: getattr(p, f) for f, _ in p._fields_})
        b = seq.encode() if isinstance(seq, str) else bytes(seq)
        return self.tiles.blat_long(b, op, max_rows)

    def caps(self, reset=True):
        from anchored_fusion_amd.blat import CAP_NAMES
        return dict(zip(CAP_NAMES, (int(v) for v in self.tiles.caps_read(reset))))

    def locate(self, t_start, t_end):
        k = bisect.bisect_right(self.offsets, int(t_start)) - 1
        if k < 0:
            return None
        s, e = int(t_start) - self.offsets[k], int(t_end) - self.offsets[k]
        if s < 0 or e > self.lens[k] or e <= s:
            return None
        return k, s, e

    def close(self):
        pass


class OracleGenomeIndex:
    """The genome calls S4 / S5 restated on the CPU (oracle/bwa_pe.c FM mode), with
    genome.GenomeIndex's interface (Searches' genome_factory)."""

    def __init__(self, contigs):
        self.g = oracle.OracleGenome(contigs)
        self.names = self.g.names

    @staticmethod
    def _params(params):
        p = oracle.default_params()
        if params is not None:
            for f, _ in p._fields_:
                setattr(p, f, getattr(params, f))
        return p

    @staticmethod
    def _pe(pe):
        e = oracle.default_pe()
        if pe is not None:
            for f, _ in e._fields_:
                setattr(e, f, getattr(pe, f))
        return e

    def align_se(self, reads, lens=None, params=None, pe=None, id_base=0):
        return self.g.align_se(reads, lens, self._params(params), self._pe(pe), id_base=id_base, threads=8)

    def align_pe(self, reads, lens=None, params=None, pe=None):
        e = self._pe(pe)
        return self.g.align_pe(reads, lens, self._params(params), e, pair_base=e.pair_base, threads=8)

    def close(self):
        pass


def oracle_searches(genome, chunk_bases=10_000_000):
    """pipeline.Searches with every service on the CPU oracles."""
    from anchored_fusion_amd import pipeline
    from anchored_fusion_amd.place import Placer
    return pipeline.Searches(genome, placer=Placer(tile_factory=OracleTileReference),
                             chunk_bases=chunk_bases, genome_factory=OracleGenomeIndex)


class OracleAligner:
    def __init__(self, anchor, chunk_bases=None):
        self.ix = oracle.OracleIndex(anchor)
        self.chunk_bases = chunk_bases

    def align_pairs(self, reads, lens=None, pair_base=0):
        o = self.ix.align_pairs(reads, lens, threads=8, pair_base=pair_base, chunk_bases=self.chunk_bases)
        return AlignResult(o["flag"], o["pos"], o["score"], o["n_cigar"], o["cigar"], o["hits"])

    def close(self):
        pass
