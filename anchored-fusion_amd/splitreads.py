"""Split-read clustering on the anchor.

Restates `contact_reads` + `combine_split_reads` (functions.py:771-952) and the record types
`Split_reads` / `Co_Split_reads` (functions.py:128-226). The input is the pseudo-SAM produced
by the genome check (a5). The output is one consensus record per breakpoint cluster.

1. **Bucket by anchor breakpoint.**
   - SM reads break at POS and need a clip of at least 15.
   - MS reads break at POS + M - 1 and are kept when the M op's running end is at least 15.
     The reference tests the running end, not the clip.
   - The bucket lookup keeps the reference's bisection, which never compares bucket 0 once a
     second bucket exists. So buckets can repeat and end up out of order, exactly as there.
   - Inside a bucket, a read joins the newest compatible record of its type. Compatible means
     the left sides agree on their common suffix and the right sides on their common prefix.
2. **Merge within a bucket.** Records merge into a per-column vote profile when both flank
   sides agree on more than 90 % of their overlap.
3. **Merge across buckets ≤ 3 nt apart** (the offset is signed). The higher-count cluster
   absorbs the other; the reference's double shift of the absorbed sequences is kept.
4. **Consensus** is the per-column majority. Ties, including empty columns, give 'N'.
"""
from .cigar import normalize

_CODE = {"A": 0, "T": 1, "G": 2, "C": 3}
_BASE = "ATGC"


class SplitRead:
    """One anchor breakpoint hypothesis (functions.py:128-157)."""
    __slots__ = ("chrom", "cnt", "breakpoint", "type_", "seq_left", "seq_right", "other_breakpoints", "reads")

    def __init__(self, chrom, breakpoint, type_, seq_left, seq_right, read):
        self.chrom, self.breakpoint, self.type_ = chrom, breakpoint, type_
        self.seq_left, self.seq_right = seq_left, seq_right
        self.cnt = 1
        self.other_breakpoints = []
        self.reads = [read]

    def add_reads(self, seq_left, seq_right, read):
        if len(seq_left) > len(self.seq_left):
            self.seq_left = seq_left
        if len(seq_right) > len(self.seq_right):
            self.seq_right = seq_right
        self.cnt += 1
        self.reads.append(read)

    def return_left_seq(self):
        return self.seq_left

    def return_right_seq(self):
        return self.seq_right

    def return_all_seq(self):
        return self.seq_left + self.seq_right

    def Add_other_breakpoint(self, chrom, breakpoint, strand, in_breakpoint, cut):  # noqa: N802 (reference name)
        self.other_breakpoints.append([chrom, breakpoint, strand, in_breakpoint, cut])

    def as_tuple(self):
        return (self.chrom, self.breakpoint, self.type_, self.seq_left, self.seq_right, self.cnt, list(self.reads))


class VoteProfile:
    """400-column base votes centred on the breakpoint (functions.py:160-226).

    Python list indexing is kept on purpose: a left flank longer than 200 wraps to the end
    of the profile and a right flank longer than 200 raises IndexError, as in the reference."""

    def __init__(self, chrom, breakpoint, type_):
        self.chrom, self.breakpoint, self.type_ = chrom, breakpoint, type_
        self.votes = [[0, 0, 0, 0] for _ in range(400)]
        self.l_left = self.l_right = 0
        self.cnt = 0
        self.reads = []

    def add(self, left, right, n, reads, shift):
        if shift >= 0:
            left, right = left + right[:shift], right[shift:]
        else:
            left, right = left[:shift], left[shift:] + right
        for off, b in enumerate(reversed(left)):
            if b in _CODE:
                self.votes[199 - off][_CODE[b]] += n
        for off, b in enumerate(right):
            if b in _CODE:
                self.votes[200 + off][_CODE[b]] += n
        self.l_left = max(self.l_left, len(left))
        self.l_right = max(self.l_right, len(right))
        self.cnt += n
        self.reads.extend(reads)

    def _call(self, col):
        v = self.votes[col]
        top = max(v)
        return "N" if v.count(top) > 1 else _BASE[v.index(top)]

    def left(self):
        return "".join(self._call(c) for c in range(200 - self.l_left, 200))

    def right(self):
        return "".join(self._call(c) for c in range(200, 200 + self.l_right))


def _agree(a, b):
    n = min(len(a), len(b))
    return sum(1 for x in range(n) if a[x] == b[x]) / n


def similar(l1, r1, l2, r2, threshold, shift):
    """functions.py:778-806: both flanks agree on more than `threshold` of their overlap,
    after moving the second pair's breakpoint by `shift`."""
    if not (l1 and l2 and r1 and r2):
        return False
    a, b = l1[::-1], l2[::-1]
    if shift >= 0:
        b = b[shift:]
    else:
        a = a[-shift:]
    if not (a and b):
        return False
    sl = _agree(a, b)
    if shift >= 0:
        r1 = r1[shift:]
    else:
        r2 = r2[-shift:]
    if not (r1 and r2):
        return False
    return sl > threshold and _agree(r1, r2) > threshold


def _bisect(buckets, bp):
    """functions.py:893-905, including that bucket 0 is only compared when it is alone."""
    lo, hi = 0, len(buckets)
    if hi == 1 and buckets[0][0] == bp:
        return True, 0
    while lo < hi - 1:
        mid = (lo + hi) // 2
        if buckets[mid][0] == bp:
            return True, mid
        if buckets[mid][0] < bp:
            lo = mid
        else:
            hi = mid
    return False, hi


def _compatible(l1, r1, l2, r2):
    n = min(len(r1), len(r2))
    return l1[max(len(l1) - len(l2), 0):] == l2[max(len(l2) - len(l1), 0):] and r1[:n] == r2[:n]


def bucket_split_reads(sam_lines):
    """Step 1 (functions.py:913-951): [(breakpoint, [SplitRead, ...]), ...] in bucket order."""
    buckets = []
    for line in sam_lines:
        f = line.split("\t")
        ops, seq = normalize(f[5], f[9])
        if len(ops) != 2:
            continue
        if ops[0][2] == "S" and ops[1][2] == "M":
            kind = "SM"
            if ops[0][0] < 15:
                continue
            bp = int(f[3])
        else:
            kind = "MS"
            if ops[1][0] < 15:
                continue
            bp = int(f[3]) + ops[0][1] - 1
        cut = ops[0][0]
        left, right = seq[:cut], seq[cut:]
        found, at = _bisect(buckets, bp)
        if not found:
            buckets.insert(at, (bp, [SplitRead(f[2], bp, kind, left, right, f[0])]))
            continue
        group = buckets[at][1]
        for rec in reversed(group):
            if rec.type_ == kind and _compatible(rec.seq_left, rec.seq_right, left, right):
                rec.add_reads(left, right, f[0])
                break
        else:
            group.append(SplitRead(f[2], bp, kind, left, right, f[0]))
    return buckets


def merge_buckets(buckets):
    """Steps 2-4 (functions.py:771-889): consensus SplitRead records."""
    profiled = []
    for bp, group in buckets:
        group = list(group)
        out = []
        while group:
            seed = group.pop(0)
            prof = VoteProfile(seed.chrom, bp, seed.type_)
            prof.add(seed.seq_left, seed.seq_right, seed.cnt, seed.reads, 0)
            rest = []
            for other in group:
                if other.type_ == seed.type_ and similar(seed.seq_left, seed.seq_right, other.seq_left,
                                                         other.seq_right, 0.9, 0):
                    prof.add(other.seq_left, other.seq_right, other.cnt, other.reads, 0)
                else:
                    rest.append(other)
            group = rest
            out.append(prof)
        profiled.append([bp, out])
    for i in range(len(profiled)):
        here = profiled[i][1]
        j = 0
        while j < len(here):
            p1 = here[j]
            l1, r1, c1, reads1, t1 = p1.left(), p1.right(), p1.cnt, p1.reads, p1.type_
            moved = False
            z = i + 1
            while not moved and z < len(profiled) and profiled[z][0] - profiled[i][0] <= 3:
                d = profiled[z][0] - profiled[i][0]
                there = profiled[z][1]
                k = 0
                while k < len(there):
                    p2 = there[k]
                    l2, r2 = p2.left(), p2.right()
                    if t1 == p2.type_ and similar(l1, r1, l2, r2, 0.9, d):
                        if c1 > p2.cnt:
                            r2, l2 = l2[-d:] + r2, l2[:-d]
                            del there[k]
                            p1.add(l2, r2, p2.cnt, p2.reads, -d)
                        else:
                            l1, r1 = l1 + r1[:d], r1[d:]
                            del here[j]
                            p2.add(l1, r1, c1, reads1, d)
                            moved = True
                            break
                    else:
                        k += 1
                z += 1
            if not moved:
                j += 1
    result = []
    for _, group in profiled:
        for p in group:
            rec = SplitRead(p.chrom, p.breakpoint, p.type_, p.left(), p.right(), "")
            rec.cnt = p.cnt
            rec.reads = p.reads
            result.append(rec)
    return result


def cluster_split_reads(sam_lines):
    """contact_reads (functions.py:892-952): pseudo-SAM lines -> consensus SplitRead list."""
    return merge_buckets(bucket_split_reads(sam_lines))
