"""Partner-gene blocks.

A block is a genomic interval of one non-homologous gene that collects evidence for the fusion
partner: spanning pairs (one mate on a homologous/anchor gene, the other on exactly one other
gene) and split-read tails placed on the genome.

* `spanning_blocks` restates the consumer side of S4, `Find_blocks` (functions.py:376-496):
  genome alignments of the one-end-anchored pairs, grouped by QNAME.
* `add_fine_blocks` restates the consumer side of S6, `Find_fine_block`
  (functions.py:506-654): PSL placements of each split read's tail.

Both insert into per-chromosome block lists kept sorted by start. A new interval joins the
block to its left when it is the same gene within that block's exon range and within 100 nt
(the two callers test that window differently; both tests are kept, `mode` picks one). Then
neighbouring blocks of the same gene merge when fewer than 200 transcript bases separate
them. The exon-walk quirks are kept: the left merge compares the exon counter with the left
block's MIN exon.
"""
import re

from .cigar import normalize


class Block:
    __slots__ = ("gene", "bad", "chrom", "start", "end", "anchored_split_breakpoints", "count", "reads",
                 "min_exon_num", "max_exon_num")

    def __init__(self, chrom, start, end, gene, exon_num):
        self.gene = gene
        self.bad = False
        self.chrom = chrom
        self.start = start
        self.end = end
        self.anchored_split_breakpoints = set()
        self.count = 0
        self.reads = []
        self.min_exon_num = exon_num
        self.max_exon_num = exon_num

    def add_read(self, start, end, read):
        self.start = min(self.start, start)
        self.end = max(self.end, end)
        self.count += 1
        self.reads.append(read)

    def absorb(self, other):
        self.start = min(self.start, other.start)
        self.end = max(self.end, other.end)
        self.count += other.count
        self.reads.extend(other.reads)
        self.min_exon_num = min(self.min_exon_num, other.min_exon_num)
        self.max_exon_num = max(self.max_exon_num, other.max_exon_num)

    def as_tuple(self):
        return (self.chrom, self.start, self.end, list(self.gene), self.count, list(self.reads),
                self.min_exon_num, self.max_exon_num)


def _gap_right(rows, left, right):
    """Transcript bases between block `left` and the block after it (functions.py:446-456)."""
    e = left.max_exon_num + 1
    gap = rows[left.max_exon_num][1] - left.end
    while e < right.min_exon_num:
        if rows[e][2] == left.gene[0] and rows[e][0] > rows[e - 1][1]:
            gap += rows[e][1] - rows[e][0]
        e += 1
    if e == right.min_exon_num:
        gap += right.start - rows[e][0]
    return gap


def _gap_left(rows, here, left):
    """Transcript bases between block `left` and block `here` (functions.py:470-479)."""
    e = here.min_exon_num - 1
    gap = here.start - rows[here.min_exon_num][0]
    while e > left.max_exon_num:
        if rows[e][2] == here.gene[0] and rows[e][1] < rows[e + 1][0]:
            gap += rows[e][1] - rows[e][0]
        e -= 1
    if e == left.min_exon_num:
        gap += rows[e][1] - left.end
    return gap


def _insert(blocks, rows, chrom, start, end, gene, exon_num, read, mode):
    i = len(blocks) - 1
    while i >= 0 and end < blocks[i].start:
        i -= 1
    join = False
    if i >= 0 and blocks[i].gene[0] == gene[0]:
        b = blocks[i]
        in_exons = b.min_exon_num <= exon_num <= b.max_exon_num
        if mode == "spanning":      # functions.py:437
            join = in_exons and start >= b.start - 100 and end <= b.end + 100
        else:                       # functions.py:569
            join = b.start - 100 <= start and b.end >= end + 100 and in_exons
    if join:
        blocks[i].add_read(start, end, read)
    else:
        nb = Block(chrom, start, end, gene, exon_num)
        nb.add_read(start, end, read)
        if i != -1 and start < blocks[i].start:
            blocks.insert(i, nb)
        else:
            i += 1
            blocks.insert(i, nb)
    # merge to the right, then to the left, while the neighbour is the same gene
    while i < len(blocks) - 1 and blocks[i].gene[0] == blocks[i + 1].gene[0]:
        here, nxt = blocks[i], blocks[i + 1]
        if nxt.min_exon_num == here.max_exon_num:
            close = here.end + 200 > nxt.start
        else:
            close = _gap_right(rows, here, nxt) <= 200
        if not close:
            break
        here.absorb(nxt)
        del blocks[i + 1]
    while i >= 1 and blocks[i].gene[0] == blocks[i - 1].gene[0]:
        here, prv = blocks[i], blocks[i - 1]
        if here.min_exon_num == prv.max_exon_num:
            close = here.start - 200 < prv.end
        else:
            close = _gap_left(rows, here, prv) <= 200
        if not close:
            break
        here.absorb(prv)
        del blocks[i - 1]
        i -= 1


def _first_match(cigar):
    """Length of the first M op and whether one exists (functions.py:377-387)."""
    m = re.search(r"(\d+)M", cigar)
    # the reference reads the digits since the previous letter: same as the \d+ run here
    return (int(m.group(1)), True) if m else (0, False)


def spanning_blocks(sam_lines, index, homo_genes):
    """S4 consumer: genome records of one-end-anchored pairs, grouped by consecutive QNAME."""
    recs = []
    for line in sam_lines:
        f = line.split("\t")
        ln, ok = _first_match(f[5])
        if ok:
            s = int(f[3])
            recs.append((f[0], f[2], s + 5, s + ln - 1 - 5))
        else:
            recs.append((f[0], "", 5, -5))
    out = {}
    j = 0
    while j < len(recs):
        k = j + 1
        while k < len(recs) and recs[k][0] == recs[j][0]:
            k += 1
        grp, j = recs[j:k], k
        if len(grp) == 1:
            continue
        coords = [c for r in grp for c in (r[2], r[3])]
        if len({r[1] for r in grp}) == 1 and max(coords) - min(coords) < 2000:
            continue
        homo_at = other_at = -1
        other_gene = other_exon = None
        for k2, (_, chrom, s, e) in enumerate(grp):
            gene, exon = index.find_exon(chrom, s, e)
            if gene[0] in homo_genes:
                homo_at = k2
            elif gene[0] != "":
                if other_at == -1:
                    other_at, other_gene, other_exon = k2, gene, exon
                elif gene[0] != other_gene[0]:
                    other_at = -1
                    break
        if homo_at == -1 or other_at == -1:
            continue
        _, chrom, s, e = grp[other_at]
        _insert(out.setdefault(chrom, []), index.dic.get(chrom), chrom, s, e, other_gene, other_exon, grp[0][0],
                "spanning")
    widen(out, index)
    return out


class S4Records:
    """S4's SAM records as `spanning_blocks` reads them, without the text: per record (in the
    order bwa prints them: read 2k's records, then read 2k + 1's) its pair, RNAME (contig index,
    -1 for '*'), POS (1-based, 0 for '*') and the length of its CIGAR's first M.  Built from the
    af_grec rows (genome.REC_DTYPE [2 P, MAX_REC]) and counts of `bwa mem -M genome tmp1 tmp2`;
    pair_names[k] is the QNAME of pair k."""

    def __init__(self, pair_names, recs, nrec, contig_names):
        import numpy as np
        nrec = np.asarray(nrec, np.int64)
        self.pair_names, self.contig_names = pair_names, list(contig_names)
        if not len(nrec):
            from .genome import REC_DTYPE
            recs = np.zeros((0, 1), REC_DTYPE)
        live = np.arange(recs.shape[1])[None, :] < np.minimum(nrec, recs.shape[1])[:, None]
        rr, kk = np.nonzero(live)
        e = recs[rr, kk]
        self.pair = rr // 2
        nc = e["n_cigar"].astype(np.int64)
        cig = e["cigar"].astype(np.int64)
        is_m = ((cig & 15) == 0) & (np.arange(cig.shape[1])[None, :] < nc[:, None])
        self.ok = is_m.any(axis=1)
        first = np.argmax(is_m, axis=1)
        self.m_len = np.where(self.ok, cig[np.arange(len(first)), first] >> 4, 0)
        rid = e["rid"].astype(np.int64)
        self.rid = np.where(self.ok, rid, -1)
        self.pos1 = np.where(rid >= 0, e["pos"].astype(np.int64) + 1, 0)
        # QNAME groups (consecutive equal names): a record starts one where its pair's name
        # differs from the previous record's
        self.group_start = np.ones(len(rr), bool)
        for t in np.flatnonzero(self.pair[1:] != self.pair[:-1]) + 1:
            self.group_start[t] = pair_names[int(self.pair[t])] != pair_names[int(self.pair[t - 1])]
        if len(rr):
            self.group_start[1:] &= self.pair[1:] != self.pair[:-1]


def spanning_blocks_records(R, index, homo_genes):
    """`spanning_blocks` over S4Records (the same blocks; the groups no rule can keep -- one
    record, or all on one contig within 2,000 nt -- are set aside vectorised)."""
    import numpy as np
    n = len(R.pair)
    out = {}
    if n:
        starts = np.flatnonzero(R.group_start)
        ends = np.r_[starts[1:], n]
        c0 = np.where(R.ok, R.pos1 + 5, 5)
        c1 = np.where(R.ok, R.pos1 + R.m_len - 1 - 5, -5)
        lo = np.minimum.reduceat(np.minimum(c0, c1), starts)
        hi = np.maximum.reduceat(np.maximum(c0, c1), starts)
        one_chrom = np.minimum.reduceat(R.rid, starts) == np.maximum.reduceat(R.rid, starts)
        keep = (ends - starts > 1) & ~(one_chrom & (hi - lo < 2000))
        names = R.contig_names
        for g in np.flatnonzero(keep):
            a, b = int(starts[g]), int(ends[g])
            homo_at = other_at = -1
            other_gene = other_exon = None
            for k2 in range(b - a):
                r = a + k2
                chrom = names[int(R.rid[r])] if R.ok[r] else ""
                gene, exon = index.find_exon(chrom, int(c0[r]), int(c1[r]))
                if gene[0] in homo_genes:
                    homo_at = k2
                elif gene[0] != "":
                    if other_at == -1:
                        other_at, other_gene, other_exon = k2, gene, exon
                    elif gene[0] != other_gene[0]:
                        other_at = -1
                        break
            if homo_at == -1 or other_at == -1:
                continue
            r = a + other_at
            chrom = names[int(R.rid[r])] if R.ok[r] else ""
            _insert(out.setdefault(chrom, []), index.dic.get(chrom), chrom, int(c0[r]), int(c1[r]), other_gene,
                    other_exon, R.pair_names[int(R.pair[a])], "spanning")
    widen(out, index)
    return out


def widen(blocks_chr, index):
    """Extend each block by 200 transcript bases on both sides (functions.py:490-495)."""
    for blocks in blocks_chr.values():
        for b in blocks:
            b.start = index.walk(b.chrom, b.start, 200)[0][0]
            b.end = index.walk(b.chrom, b.end, 200)[-1][1]


class _Tail:
    __slots__ = ("kind", "left", "right", "name")

    def __init__(self, kind, left, right, name):
        self.kind, self.left, self.right, self.name = kind, left, right, name


def split_read_queries(sam_lines):
    """The FASTA that S6 sends to BLAT (functions.py:512-528): ordinal ids, processed seqs."""
    tails, fasta = [], []
    for line in sam_lines:
        f = line.split("\t")
        ops, seq = normalize(f[5], f[9])
        if len(ops) != 2:
            continue
        kind = "SM" if (ops[0][2] == "S" and ops[1][2] == "M") else "MS"
        fasta.append((str(len(tails)), seq))
        tails.append(_Tail(kind, ops[0][1], ops[1][1], f[0]))
    return tails, fasta


def add_fine_blocks(blocks_chr, tails, psl_lines, index, homo_genes):
    """S6 consumer (functions.py:531-649): PSL placements grouped by query id.

    A query group contributes its `blocks` candidates when some placement showed the anchored
    half on a homologous gene (`good`) and no placement covered both halves (`bad`).  As in
    the reference, the good/bad state is only reset after a rejected group.
    """
    bad = good = 0
    pending = []
    last = -1

    def flush():
        for chrom, s, e, name in pending:
            gene, exon = index.find_exon(chrom, s, e)
            if gene[0] == "" or gene[0] in homo_genes:
                continue
            if chrom not in blocks_chr:
                nb = Block(chrom, s, e, gene, exon)
                nb.add_read(s, e, name)
                blocks_chr[chrom] = [nb]
            else:
                _insert(blocks_chr[chrom], index.dic.get(chrom), chrom, s, e, gene, exon, name, "fine")

    rows = [ln.split("\t") for ln in psl_lines if re.match(r"^\d+\s", ln)]
    for f in rows + [None]:
        qid = int(f[9]) if f is not None else -2
        if qid != last:
            last = qid
            if bad == 1 or good == 0:
                bad = good = 0
            else:
                flush()
            pending = []
        if bad != 0 or f is None:
            continue
        chrom, s, e, qs, qe = f[13], int(f[15]), int(f[16]), int(f[11]), int(f[12])
        if e - s > 200:
            continue
        t = tails[qid]
        L, R = t.left, t.right
        if t.kind == "MS":
            if qs <= L // 2 and qe >= L + 5:
                bad = 1
            elif L - 5 <= qs <= L + 5 and qe >= L + R - 5:
                pending.append((chrom, s, e, t.name))
            elif qs <= 5 and qe <= L + 5:
                if index.find_exon(chrom, s, e)[0][0] in homo_genes:
                    good = 1
        else:
            if L - 5 <= qe <= L + 5 and qs <= 5:
                pending.append((chrom, s, e, t.name))
            elif qs < L - 5 and qe >= L + R // 2:
                bad = 1
            elif L - 5 <= qs <= L + 5 and qe >= L + R - 5:
                if index.find_exon(chrom, s, e)[0][0] in homo_genes:
                    good = 1
    return blocks_chr
