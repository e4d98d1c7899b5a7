"""Long BLAT queries as one stitched alignment (functions.py:341 `Find_homo_genes`, fn:966).

The reference hands BLAT the whole anchor transcript (kilobases) as one query; BLAT cuts a long
query into overlapping pieces, finds each piece's alignments and stitches the colinear ones of
one target back into a single alignment (blocks across the introns), and only then applies
-minScore / -minIdentity (Kent 2002; blat's long-DNA path).  The search kernel takes queries of
at most AF_MAX_READ bases, so a long query is searched as WINDOW-base windows at a WINDOW / 2
step with no score / identity floor (the kernel's tile, clump and extension rules unchanged),
and this module stitches the window alignments with the restatement's own chaining rule
(oracle/blat.c `blat_strand`, csrc/blat.hip): per strand, alignments ordered by (qStart, tStart,
qEnd); an alignment follows another when it ends later on both sequences; its front is trimmed
until it starts after the other on both; the target gap is at most max_intron without an N
between; chain score = sum of the parts' matches - mismatches - inserts, minus one per query and
per target gap between parts; best chain first, its parts then used up together with every
alignment sharing an aligned column with it (the overlapping windows' views of the same
alignment).  The stitched row
(abutting blocks merged, counts recomputed from the bases) passes when its score reaches
min_score and its milliBad (psl_millibad, mRNA form) is within 10 * (100 - min_identity).

Host code over the kernel's rows: a handful of long queries per gene (the anchor), not the
per-read hot path.  Parity with the BLAT binary stays unpinned (SURVEY.md §8 c).
"""
import math
import re

import numpy as np

WINDOW = 300
_NON_ACGT = re.compile("[^ACGTacgt]")
_COMP = str.maketrans("ACGTNacgtn", "TGCANtgcan")
_CODE = np.full(256, 4, np.int8)
for _i, _c in enumerate(b"ACGT"):
    _CODE[_c] = _i
    _CODE[_c + 32] = _i


def windows(seq):
    """(offset, window) pieces of a long query: WINDOW bases at a WINDOW // 2 step, the last
    window ending at the query's end."""
    step = WINDOW // 2
    out = []
    for off in range(0, max(1, len(seq) - step), step):
        out.append((off, seq[off:off + WINDOW]))
    return out


class _Part:
    """One window alignment in whole-query coordinates of its strand: aligned columns (q, t)
    with per-column class (0 match, 1 mismatch, 2 N) and block index, prefix sums for trims."""

    def __init__(self, strand, tk, blocks, Q, T):
        self.strand, self.tk = strand, tk
        q = np.concatenate([np.arange(b[0], b[0] + b[2]) for b in blocks])
        t = np.concatenate([np.arange(b[1], b[1] + b[2]) for b in blocks])
        blk = np.concatenate([np.full(b[2], k) for k, b in enumerate(blocks)])
        qc = _CODE[np.frombuffer(Q, np.uint8)[q]]
        tc = _CODE[np.frombuffer(T[int(t[0]):int(t[-1]) + 1].encode(), np.uint8)[t - t[0]]]
        cls = np.where((qc > 3) | (tc > 3), 2, np.where(qc == tc, 0, 1))
        self.q, self.t, self.blk = q, t, blk
        self.keys = (t.astype(np.int64) << 20) | q  # aligned columns (query < 2^20)
        self.cum = np.zeros((3, len(q) + 1), np.int64)
        for c in range(3):
            self.cum[c, 1:] = np.cumsum(cls == c)
        # gaps after block k (k -> k + 1): query / target insert counts and bases, suffix sums
        nb = len(blocks)
        g = np.zeros((4, nb + 1), np.int64)
        for k in range(nb - 1):
            qg = blocks[k + 1][0] - (blocks[k][0] + blocks[k][2])
            tg = blocks[k + 1][1] - (blocks[k][1] + blocks[k][2])
            g[:, k] = (qg > 0, max(qg, 0), tg > 0, max(tg, 0))
        self.gsuf = np.cumsum(g[:, ::-1], axis=1)[:, ::-1]  # gsuf[:, k] = gaps after blocks k..
        self.qe, self.te = int(q[-1]) + 1, int(t[-1]) + 1
        self.qb, self.tb = int(q[0]), int(t[0])

    def cut(self, qe, te):
        """first column starting at or after (qe, te) on both sequences (len(q): none)"""
        return max(int(np.searchsorted(self.q, qe)), int(np.searchsorted(self.t, te)))

    def stats(self, c):
        n = len(self.q)
        m, x, nc = (int(self.cum[k, n] - self.cum[k, c]) for k in range(3))
        qni, qbi, tni, tbi = (int(v) for v in self.gsuf[:, int(self.blk[c])])
        return m, x, nc, qni, qbi, tni, tbi

    def score(self, c):
        m, x, _, qni, _, tni, _ = self.stats(c)
        return m - x - qni - tni

    def blocks(self, c):
        out = []
        q, t, blk = self.q[c:], self.t[c:], self.blk[c:]
        starts = np.flatnonzero(np.r_[True, blk[1:] != blk[:-1]])
        ends = np.r_[starts[1:], len(q)]
        for s, e in zip(starts, ends):
            out.append([int(q[s]), int(t[s]), int(e - s)])
        return out


def _millibad(q_ali, t_ali, m, x, qni):
    if min(q_ali, t_ali) <= 0:
        return 0
    dif = max(q_ali - t_ali, 0)
    total = m + x
    if total == 0:
        return 0
    return int((1000 * (x + qni + round(3 * math.log(1.0 + dif)))) // total)


def stitch(parts, T, L, p):
    """Chains of one strand and target contig (text T, str) -> PSL rows (dicts) that pass."""
    parts = sorted(parts, key=lambda a: (a.qb, a.tb, a.qe))
    n = len(parts)
    used = [False] * n
    out = []
    while True:
        best, prev = [0] * n, [-1] * n
        bi = -1
        for i in range(n):
            if used[i]:
                continue
            b = parts[i]
            best[i] = b.score(0)
            for j in range(i):
                if used[j]:
                    continue
                a = parts[j]
                if b.qe <= a.qe or b.te <= a.te:
                    continue
                c = b.cut(a.qe, a.te)
                if c >= len(b.q):
                    continue
                tb = int(b.t[c])
                if tb - a.te > p.max_intron or _NON_ACGT.search(T, a.te, tb):
                    continue
                s = best[j] + b.score(c) - (int(b.q[c]) > a.qe) - (tb > a.te)
                if s > best[i]:
                    best[i], prev[i] = s, j
            if bi < 0 or best[i] > best[bi]:
                bi = i
        if bi < 0 or best[bi] < p.min_score:
            break  # scores only fall as parts are used up
        chain = []
        i = bi
        while i >= 0:
            chain.append(i)
            i = prev[i]
        chain.reverse()
        blocks, tot = [], np.zeros(7, np.int64)
        for k, i in enumerate(chain):
            used[i] = True
            a = parts[chain[k - 1]] if k else None
            c = parts[i].cut(a.qe, a.te) if a is not None else 0
            tot += parts[i].stats(c)
            bl = parts[i].blocks(c)
            if a is not None:
                qg, tg = bl[0][0] - a.qe, bl[0][1] - a.te
                tot += (0, 0, 0, qg > 0, max(qg, 0), tg > 0, max(tg, 0))
            for blk in bl:
                last = blocks[-1] if blocks else None
                if last and last[0] + last[2] == blk[0] and last[1] + last[2] == blk[1]:
                    last[2] += blk[2]
                else:
                    blocks.append(blk)
        # the other windows' views of the same alignment (a shared aligned column) are used up too
        keys = np.concatenate([parts[i].keys for i in chain])
        for j in range(n):
            if not used[j] and np.isin(parts[j].keys, keys).any():
                used[j] = True
        m, x, nc, qni, qbi, tni, tbi = (int(v) for v in tot)
        score = m - x - qni - tni
        qb, qe = blocks[0][0], blocks[-1][0] + blocks[-1][2]
        tb, te = blocks[0][1], blocks[-1][1] + blocks[-1][2]
        if _millibad(qe - qb, te - tb, m, x, qni) > (100 - p.min_identity) * 10:
            continue
        strand = parts[bi].strand
        out.append(dict(score=score, strand=strand, m=m, x=x, nc=nc, qni=qni, qbi=qbi, tni=tni, tbi=tbi,
                        q_start=L - qe if strand else qb, q_end=L - qb if strand else qe, t_start=tb, t_end=te,
                        blocks=blocks))
    return out


def stitched_lines(ref, targets, name, seq, rows, nr, pieces, p):
    """PSL lines of the long query (name, seq) from the window rows `rows[i]` / `nr[i]` of its
    pieces [(offset, window)], sorted as the kernel sorts a query's rows (score desc, strand,
    target start, query start, target end, query end)."""
    L = len(seq)
    fwd = seq.upper()
    strand_q = (fwd.encode(), fwd.translate(_COMP)[::-1].encode())
    seen, groups = set(), {}
    for (off, w), rr, n in zip(pieces, rows, nr):
        for k in range(max(int(n), 0)):
            r = rr[k]
            loc = ref.locate(r["t_start"], r["t_end"])
            if loc is None:
                continue
            tk = loc[0]
            base = ref.offsets[tk]
            s = int(r["strand"])
            shift = L - (off + len(w)) if s else off
            nb = int(r["block_count"])
            blocks = tuple((shift + int(r["q_starts"][b]), int(r["t_starts"][b]) - base, int(r["block_sizes"][b]))
                           for b in range(nb))
            if not nb or (s, tk, blocks) in seen:
                continue
            seen.add((s, tk, blocks))
            groups.setdefault((s, tk), []).append(blocks)
    found = []
    for (s, tk), bls in groups.items():
        T = targets[tk][1]
        T = T if isinstance(T, str) else bytes(T).decode()
        parts = [_Part(s, tk, b, strand_q[s], T) for b in bls]
        for row in stitch(parts, T, L, p):
            found.append((tk, row))
    found.sort(key=lambda e: (-e[1]["score"], e[1]["strand"], ref.offsets[e[0]] + e[1]["t_start"], e[1]["q_start"],
                              ref.offsets[e[0]] + e[1]["t_end"], e[1]["q_end"]))
    out = []
    for tk, r in found:
        bl = r["blocks"]
        f = [r["m"], r["x"], 0, r["nc"], r["qni"], r["qbi"], r["tni"], r["tbi"], "-" if r["strand"] else "+", name, L,
             r["q_start"], r["q_end"], ref.names[tk], ref.lens[tk], r["t_start"], r["t_end"], len(bl),
             ",".join(str(b[2]) for b in bl) + ",", ",".join(str(b[0]) for b in bl) + ",",
             ",".join(str(b[1]) for b in bl) + ","]
        out.append("\t".join(map(str, f)) + "\n")
    return out
