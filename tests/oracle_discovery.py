"""The CPU oracle as a backend of anchored_fusion_amd.dist_discover -- TEST INFRASTRUCTURE ONLY.

The three phases of a rank (S2 + S3 + the gathers; S4 on whole chunks of its stream; S5 with the given read ids,
its genome check with the given QNAME groups, S6) computed by oracle/bwa_pe.c, oracle/blat.c and
the host restatements the consumer stages use (align.partition, genome_check, blocks), so the
distributed driver can be checked on CPU with gloo against the one-process host path."""
import numpy as np

ALL_ROWS = 256  # rows per S6 query the oracle backend keeps (the GPU: MAX_ROWS + its spill pool)

import afpkg  # noqa: F401
import oracle
from anchored_fusion_amd import blat, blocks, genome, genome_check
from anchored_fusion_amd.align import AlignResult, partition
from anchored_fusion_amd.cigar import normalize
from anchored_fusion_amd.dist_discover import LocalQueries, cigar_string
from oracle_backends import OracleTileReference

_COMP = bytes.maketrans(b"ACGTN", b"TGCAN")


class OracleDiscovery:
    def __init__(self, anchor, og, tiles, reads, lens, pair_base, chunk_bases, gene):
        self.ix = oracle.OracleIndex(anchor)
        self.og, self.tiles = og, tiles
        self.reads, self.pair_base, self.chunk_bases, self.gene = reads, int(pair_base), int(chunk_bases), gene
        self.lens = np.full(reads.shape[0], reads.shape[1], np.int32) if lens is None else np.asarray(lens, np.int32)

    def _seq(self, r):
        return self.reads[r, :self.lens[r]]

    def local_phase(self):
        o = self.ix.align_pairs(self.reads, self.lens, threads=8, pair_base=self.pair_base,
                                chunk_bases=self.chunk_bases)
        res = AlignResult(o["flag"], o["pos"], o["score"], o["n_cigar"], o["cigar"], o["hits"])
        self.res = res
        t1, t2, an = partition(res)

        def key(rows):
            rows = np.asarray(rows, np.int64)
            return res.pos[rows].astype(np.int64) * 2 + ((res.flag[rows] & 0x10) != 0)

        def seq_list(rows):
            rows = np.asarray(rows, np.int64)
            return self.reads[rows], self.lens[rows]
        s1, l1 = seq_list(t1)
        s2, l2 = seq_list(t2)
        rows5, seqs5 = [], []
        for r in an:
            s = self._seq(int(r)).tobytes()
            if len(normalize(res.cigar_str(r), s.decode())[0]) == 2:
                rows5.append(int(r))
                seqs5.append(s[::-1].translate(_COMP) if res.flag[r] & 0x10 else s)
        rows5 = np.asarray(rows5, np.int64)
        self.q5 = seqs5
        self._cig = res.cigar[rows5] if len(rows5) else np.zeros((0, 32), np.uint32)
        self._ncig = res.n_cigar[rows5] if len(rows5) else np.zeros(0, np.int32)
        return LocalQueries(
            dict(key=key(t1), row=np.asarray(t1, np.int64), seq=s1, len=l1),
            dict(key=key(t2), row=np.asarray(t2, np.int64), seq=s2, len=l2),
            dict(key=key(rows5), row=rows5, pos=res.pos[rows5] if len(rows5) else np.zeros(0, np.int32),
                 ncig=res.n_cigar[rows5] if len(rows5) else np.zeros(0, np.int32),
                 cigar=(res.cigar[rows5] if len(rows5) else np.zeros((0, 32), np.uint32)).view(np.int32),
                 seq=_rows([np.frombuffer(x, np.uint8) for x in seqs5]),
                 len=np.array([len(x) for x in seqs5], np.int32)))

    def s4_phase(self, q, ql, pair_base=0):
        pe = oracle.default_pe(chunk_bases=self.chunk_bases)
        recs, nrec = self.og.align_pe(_np(q), _np(ql).astype(np.int32), pe=pe, pair_base=pair_base, threads=8)
        return recs.view(np.int32).reshape(recs.shape[0], recs.shape[1], -1), nrec

    def s5_s6_phase(self, ids, cont):
        ids, cont = _np(ids), _np(cont)
        n5 = len(self.q5)
        out = dict(src=np.zeros(0, np.int64), s6_seq=np.zeros((0, 1), np.uint8), s6_len=np.zeros(0, np.int32),
                   psl=np.zeros((0, blat.MAX_ROWS, 82), np.int32), n_psl=np.zeros(0, np.int32))
        if not n5:
            return out
        buf = np.full((n5, max(len(s) for s in self.q5)), ord("N"), np.uint8)
        ql = np.zeros(n5, np.int32)
        for i, s in enumerate(self.q5):
            buf[i, :len(s)] = np.frombuffer(s, np.uint8)
            ql[i] = len(s)
        recs, nrec = self.og.align_se(buf, ql, ids=ids, threads=8)
        gid = np.zeros(n5, np.int64)
        for i in range(n5):
            gid[i] = gid[i - 1] if (i and cont[i]) else i
        # the check over the SAM text, grouped as the caller says: a group's queries share a
        # QNAME (its first query's index; the check reads only the QNAME's CIGAR field)
        lines = ["@HD\tVN:1.6\n"]
        for i in range(n5):
            name = f"{gid[i]}${self.gene}$0${cigar_string(self._cig[i], self._ncig[i])}"
            lines += genome.sam_lines(self.og.names, name, self.q5[i].decode(), recs[i], nrec[i])
        split = genome_check.filter_genome_hits(lines)
        _, fa = blocks.split_read_queries(split)
        out["src"] = np.array([int(ln.split("\t")[0]) for ln in split], np.int64)
        seqs = [sq for _, sq in fa]
        out["s6_seq"] = _rows([np.frombuffer(x.encode(), np.uint8) for x in seqs])
        out["s6_len"] = np.array([len(x) for x in seqs], np.int32)
        if fa:
            # every row (up to ALL_ROWS): the first MAX_ROWS kept, the rest as the GPU's spill pool
            allr, alln = self.tiles.search(seqs, blat.params("split_tail"), ALL_ROWS)
            M = blat.MAX_ROWS
            out["n_psl"] = np.minimum(alln, M).astype(np.int32)
            out["psl"] = np.ascontiguousarray(allr[:, :M]).view(np.int32).reshape(len(seqs), M, -1)
            sq = np.concatenate([np.full(max(0, int(c) - M), k, np.int64) for k, c in enumerate(alln)] +
                                [np.zeros(0, np.int64)])
            sr = np.concatenate([allr[k, M:int(c)] for k, c in enumerate(alln)] + [allr[:0, 0]])
            out["spill_q"] = sq
            out["spill_psl"] = np.ascontiguousarray(sr).view(np.int32).reshape(len(sr), blat.PSL_DTYPE.itemsize // 4)
        return out

    def psl_lines(self, queries, rows, nrows, extra=None):
        return blat.psl_lines(self.tiles, queries, np.stack(rows), np.asarray(nrows), extra=extra)


def _np(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


def _rows(seqs):
    """Sequences (uint8 arrays) as one uint8 [k, w] block ('N' padded)."""
    out = np.full((len(seqs), max([1] + [len(x) for x in seqs])), ord("N"), np.uint8)
    for i, x in enumerate(seqs):
        out[i, :len(x)] = x
    return out


def tiles_for(genome_contigs):
    return OracleTileReference(genome_contigs, blat.params("split_tail").step_size)
