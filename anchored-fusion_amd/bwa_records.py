"""The SAM records `bwa mem -M` prints for the genome searches, from the placement hits.

The reference runs bwa against the genome twice:

- S4, paired: `bwa mem -M -t T genome tmp1.fq tmp2.fq` (Anchored_Fusion.py:188), consumed by
  `Find_blocks` (functions.py:376-496), which reads every record of a QNAME;
- S5, single-end: `bwa mem -M -t T genome split.fa` (functions.py:716), consumed by
  `del_too_many_reads` (fn:705-768), which reads every record of a query, turns its first `H` into
  `S` and reverse-complements SEQ for 0x10.

The GPU placement (`af_place`, place.py) returns every seed-extended region scoring >= T per
query.  This module restates what bwa 0.7.17 prints from such a region list (bwamem.c,
bwamem_pair.c; the same routines oracle/bwa_pe.c restates for S2):

- `mark_primary_se` (mem_mark_primary_se): regions ordered by score, ties by hash_64(id + i); a
  region overlapping a better one by >= mask_level (0.5) of the shorter query span is secondary;
- `mem_reg2sam` with -M: the primary, then every other non-secondary region >= T as a 0x100 record
  (bwa's supplementary 0x800 under -M) with hard clips and SEQ trimmed to the aligned part;
  secondaries go to XA (not a record); no region >= T -> one unmapped record;
- `mem_sam_pe` for S4: insert-size statistics of the run's chunks (mem_pestat), mem_pair's choice
  of the best-scoring consistent pair (its hash_64 tie-break included), the proper-pair flag, the
  chimeric (is_multi) and unpaired-score fallbacks, and the mate fields of mem_aln2sam.

Not restated: mate rescue (mem_matesw) against the genome -- a pair whose orientation statistics
succeed and whose mate has no region of its own is left unrescued -- and MAPQ (printed as 60; no
consumer reads it).  Regions come from the placement engine, capped at 16 per query (bwa keeps
all); the region set itself is the engine's, bit-exact vs the oracle (af_place / afo_place).
"""
import math

from .align import chunk_ends

MASK_LEVEL = 0.5       # mem_opt_t.mask_level
MIN_RATIO = 0.8        # bwamem_pair.c
MIN_DIR_CNT = 10
MIN_DIR_RATIO = 0.05
OUTLIER_BOUND = 2.0
MAPPING_BOUND = 3.0
MAX_STDDEV = 4.0
PEN_UNPAIRED = 17      # -U
MAX_INS = 10000
CHUNK_BASES = 10_000_000
M64 = (1 << 64) - 1
_OPS = "MIDNSHP=X"
_COMP = str.maketrans("ACGTNacgtn", "TGCANtgcan")


def hash_64(key):
    """bwa utils.h hash_64 (64-bit wrap-around)."""
    key &= M64
    key = (key + (~(key << 32) & M64)) & M64
    key ^= key >> 22
    key = (key + (~(key << 13) & M64)) & M64
    key ^= key >> 8
    key = (key + (key << 3)) & M64
    key ^= key >> 15
    key = (key + (~(key << 27) & M64)) & M64
    key ^= key >> 31
    return key


class Region:
    """One placement hit as a bwa mem_alnreg_t: query span [qb, qe) on the read as given, reference
    span [rb, re) on bwa's doubled text (reverse-strand hits at 2 l_pac - end), the contig."""
    __slots__ = ("score", "qb", "qe", "rb", "re", "rid", "rev", "k", "secondary", "sub", "hash")

    def __init__(self, score, qb, qe, rb, re, rid, rev, k):
        self.score, self.qb, self.qe, self.rb, self.re = score, qb, qe, rb, re
        self.rid, self.rev, self.k = rid, rev, k
        self.secondary, self.sub, self.hash = -1, 0, 0


def regions(ref, hits_row, n):
    """Regions of one query's hits, in mem_sort_dedup_patch order (score desc, rb, qb)."""
    l_pac = ref.total
    out = []
    for k in range(max(int(n), 0)):
        h = hits_row[k]
        loc = ref.locate(h["t_start"], h["t_end"])
        if loc is None:
            continue
        ts, te = int(h["t_start"]), int(h["t_end"])
        rev = bool(int(h["flag"]) & 0x10)
        rb, re_ = (2 * l_pac - te, 2 * l_pac - ts) if rev else (ts, te)
        out.append(Region(int(h["score"]), int(h["q_start"]), int(h["q_end"]), rb, re_, loc[0], rev, k))
    out.sort(key=lambda r: (-r.score, r.rb, r.qb))
    return out


def _overlap_secondary(regs):
    """mem_mark_primary_se_core over regs (already in score / hash order)."""
    z = [0] if regs else []
    for i in range(1, len(regs)):
        a_i = regs[i]
        for j in z:
            a_j = regs[j]
            b_max, e_min = max(a_j.qb, a_i.qb), min(a_j.qe, a_i.qe)
            if e_min > b_max:
                min_l = min(a_i.qe - a_i.qb, a_j.qe - a_j.qb)
                if e_min - b_max >= min_l * MASK_LEVEL:
                    if a_j.sub == 0:
                        a_j.sub = a_i.score
                    a_i.secondary = j
                    break
        else:
            z.append(i)


def mark_primary_se(regs, read_id):
    """mem_mark_primary_se: returns regs reordered (score desc, hash_64(id + i) asc) with
    .secondary set (-1 for a primary or chimeric part)."""
    for i, r in enumerate(regs):
        r.sub, r.secondary, r.hash = 0, -1, hash_64(read_id + i)
    out = sorted(regs, key=lambda r: (-r.score, r.hash))
    _overlap_secondary(out)
    return out


def _cigar_ops(h):
    return [(int(c) >> 4, int(c) & 15) for c in h["cigar"][:int(h["n_cigar"])]]


def _record(ref, name, seq, h, r, flag, supp, rnext="*", pnext=0):
    """One mapped SAM line (mem_aln2sam): a supplementary part (-M: 0x100) gets hard clips and the
    clipped SEQ; SEQ is reverse-complemented for 0x10."""
    ops = _cigar_ops(h)
    s = seq.translate(_COMP)[::-1] if r.rev else seq
    if supp:
        qb, qe = 0, len(s)
        if ops and ops[0][1] == 4:
            qb = ops[0][0]
            ops[0] = (ops[0][0], 5)
        if ops and ops[-1][1] == 4:
            qe -= ops[-1][0]
            ops[-1] = (ops[-1][0], 5)
        s = s[qb:qe]
    cig = "".join(f"{n}{_OPS[o]}" for n, o in ops)
    _, ts, _ = ref.locate(h["t_start"], h["t_end"])
    return f"{name}\t{flag}\t{ref.names[r.rid]}\t{ts + 1}\t60\t{cig}\t{rnext}\t{pnext}\t0\t{s}\t*\n"


class Mate:
    """The other end's printed alignment for mem_aln2sam's mate fields (rname None: unmapped)."""
    __slots__ = ("rname", "pos", "rev")

    def __init__(self, rname=None, pos=0, rev=False):
        self.rname, self.pos, self.rev = rname, pos, rev


def _mate_fields(flag, rname, pos1, rev, m):
    """mem_aln2sam's paired flag / RNEXT / PNEXT rules: an unmapped end takes its mapped mate's
    place and strand, a mapped end with an unmapped mate lends it its own."""
    flag |= 0x1
    if m.rname is None:
        flag |= 0x8
        if rname is not None:
            flag |= 0x20 if rev else 0
            return flag, "=", pos1
        return flag, "*", 0
    flag |= 0x20 if m.rev else 0
    if rname is None:
        flag |= 0x10 if m.rev else 0
        return flag, "=", m.pos
    return flag, ("=" if m.rname == rname else m.rname), m.pos


def se_records(ref, name, seq, hits_row, n, read_id, T, extra_flag=0, mate=None, regs=None):
    """mem_reg2sam (-M) for one read: its SAM lines, primary first.  mate (Mate): the other end for
    paired output, else None (single-end)."""
    if regs is None:
        regs = mark_primary_se(regions(ref, hits_row, n), read_id)
    out = []
    for r in regs:
        if r.score < T or r.secondary >= 0:
            continue
        supp = len(out) > 0
        flag = extra_flag | (0x10 if r.rev else 0) | (0x100 if supp else 0)
        rnext, pnext = "*", 0
        if mate is not None:
            _, ts, _ = ref.locate(hits_row[r.k]["t_start"], hits_row[r.k]["t_end"])
            flag, rnext, pnext = _mate_fields(flag, ref.names[r.rid], ts + 1, r.rev, mate)
        out.append(_record(ref, name, seq, hits_row[r.k], r, flag, supp, rnext, pnext))
    if not out:
        flag, rname, pos, rnext, pnext = 4 | extra_flag, "*", 0, "*", 0
        if mate is not None:
            flag, rnext, pnext = _mate_fields(flag, None, 0, False, mate)
            if mate.rname is not None:  # placed at its mapped mate
                rname, pos = mate.rname, mate.pos
        out.append(f"{name}\t{flag}\t{rname}\t{pos}\t0\t*\t{rnext}\t{pnext}\t0\t{seq}\t*\n")
    return out


# ---------------------------------------------------------------------------- paired end
def _cal_sub(regs):
    for j in range(1, len(regs)):
        b_max, e_min = max(regs[j].qb, regs[0].qb), min(regs[j].qe, regs[0].qe)
        if e_min > b_max:
            min_l = min(regs[j].qe - regs[j].qb, regs[0].qe - regs[0].qb)
            if e_min - b_max >= min_l * MASK_LEVEL:
                return regs[j].score
    return None


def infer_dir(l_pac, b1, b2):
    """mem_infer_dir -> (orientation 0..3, distance)."""
    r1, r2 = b1 >= l_pac, b2 >= l_pac
    p2 = b2 if r1 == r2 else 2 * l_pac - 1 - b2
    dist = p2 - b1 if p2 > b1 else b1 - p2
    return (0 if r1 == r2 else 1) ^ (0 if p2 > b1 else 3), dist


class PeStat:
    __slots__ = ("low", "high", "failed", "avg", "std")

    def __init__(self):
        self.low = self.high = 0
        self.failed, self.avg, self.std = 0, 0.0, 0.0


def pestat(pair_regs, l_pac, min_seed_len=19, a=1):
    """mem_pestat over one chunk's pairs [(regs1, regs2)] (regions in mem_sort_dedup_patch order)."""
    isz = [[], [], [], []]
    for r0, r1 in pair_regs:
        if not r0 or not r1:
            continue
        s0, s1 = _cal_sub(r0), _cal_sub(r1)
        if (s0 if s0 is not None else min_seed_len * a) > MIN_RATIO * r0[0].score:
            continue
        if (s1 if s1 is not None else min_seed_len * a) > MIN_RATIO * r1[0].score:
            continue
        if r0[0].rid != r1[0].rid:
            continue
        d, dist = infer_dir(l_pac, r0[0].rb, r1[0].rb)
        if dist and dist <= MAX_INS:
            isz[d].append(dist)
    pes = [PeStat() for _ in range(4)]
    for d in range(4):
        r, q = pes[d], sorted(isz[d])
        n = len(q)
        if n < MIN_DIR_CNT:
            r.failed = 1
            continue
        p25, p75 = q[int(.25 * n + .499)], q[int(.75 * n + .499)]
        r.low = max(1, int(p25 - OUTLIER_BOUND * (p75 - p25) + .499))
        r.high = int(p75 + OUTLIER_BOUND * (p75 - p25) + .499)
        kept = [v for v in q if r.low <= v <= r.high]
        avg = 0.0
        for v in kept:
            avg += v
        avg /= len(kept)
        sd = 0.0
        for v in kept:
            sd += (v - avg) * (v - avg)
        sd = math.sqrt(sd / len(kept))
        r.avg, r.std = avg, sd
        r.low = int(p25 - MAPPING_BOUND * (p75 - p25) + .499)
        r.high = int(p75 + MAPPING_BOUND * (p75 - p25) + .499)
        if r.low > avg - MAX_STDDEV * sd:
            r.low = int(avg - MAX_STDDEV * sd + .499)
        if r.high < avg + MAX_STDDEV * sd:
            r.high = int(avg + MAX_STDDEV * sd + .499)
        r.low = max(1, r.low)
    mx = max(len(v) for v in isz)
    for d in range(4):
        if not pes[d].failed and len(isz[d]) < mx * MIN_DIR_RATIO:
            pes[d].failed = 1
    return pes


def _to_i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


def mem_pair(regs, pes, pair_id, l_pac, ref, p_a=1, tmp=5 + 1 + 6):
    """mem_pair over the two mates' marked regions -> (score, (z0, z1)) or (0, None)."""
    v = []
    for r in range(2):
        for i, e in enumerate(regs[r]):
            x = e.rb if e.rb < l_pac else 2 * l_pac - 1 - e.rb
            x = (e.rid << 32) | (x - ref.offsets[e.rid])
            y = (e.score << 32) | (i << 2) | ((1 if e.rb >= l_pac else 0) << 1) | r
            v.append((x, y))
    v.sort()
    y = [-1, -1, -1, -1]
    u = []
    idk = _to_i32((pair_id & 0xFFFFFFFF) << 8) & M64
    for i in range(len(v)):
        for r in range(2):
            d = r << 1 | (v[i][1] >> 1 & 1)
            if pes[d].failed:
                continue
            which = r << 1 | ((v[i][1] & 1) ^ 1)
            if y[which] < 0:
                continue
            for k in range(y[which], -1, -1):
                if (v[k][1] & 3) != which:
                    continue
                dist = v[i][0] - v[k][0]
                if dist > pes[d].high:
                    break
                if dist < pes[d].low:
                    continue
                ns = (dist - pes[d].avg) / pes[d].std
                q = int((v[i][1] >> 32) + (v[k][1] >> 32)
                        + .721 * math.log(2. * math.erfc(abs(ns) * math.sqrt(0.5))) * p_a + .499)
                q = max(q, 0)
                key_y = (k << 32) | i
                u.append(((q << 32) | (hash_64(key_y ^ idk) & 0xFFFFFFFF), key_y))
        y[v[i][1] & 3] = i
    if not u:
        return 0, None
    u.sort()
    i, k = u[-1][1] >> 32, u[-1][1] & 0xFFFFFFFF
    z = [0, 0]
    z[v[i][1] & 1] = (v[i][1] & 0xFFFFFFFF) >> 2
    z[v[k][1] & 1] = (v[k][1] & 0xFFFFFFFF) >> 2
    return u[-1][0] >> 32, tuple(z)


def pe_records(ref, pairs, hits, nh, T, min_seed_len=19, chunk_bases=CHUNK_BASES):
    """`bwa mem -M genome fq1 fq2` records for pairs [(qname, seq1, seq2)] placed as
    hits[2i], hits[2i + 1] (rows of af_place output).  Returns SAM lines, per pair mate 1's
    records then mate 2's, as bwa prints them."""
    l_pac = ref.total
    raw = [(regions(ref, hits[2 * i], nh[2 * i]), regions(ref, hits[2 * i + 1], nh[2 * i + 1]))
           for i in range(len(pairs))]
    ends = chunk_ends([len(a) + len(b) for _, a, b in pairs], chunk_bases) if pairs else []
    out, start = [], 0
    for end in ends:
        pes = pestat(raw[start:end], l_pac, min_seed_len)
        for i in range(start, end):
            out += _sam_pe(ref, pairs[i], hits[2 * i], hits[2 * i + 1], raw[i], pes, i, T, l_pac)
        start = end
    return out


def _sam_pe(ref, pair, h0, h1, raw, pes, pid, T, l_pac):
    """mem_sam_pe without mate rescue (module docstring)."""
    name, s0, s1 = pair
    a = [mark_primary_se(list(raw[0]), pid << 1 | 0), mark_primary_se(list(raw[1]), pid << 1 | 1)]
    seqs, hs = (s0, s1), (h0, h1)

    def mate_of(i, r):
        if r is None:
            return Mate()
        _, ts, _ = ref.locate(hs[i][r.k]["t_start"], hs[i][r.k]["t_end"])
        return Mate(ref.names[r.rid], ts + 1, r.rev)
    if a[0] and a[1]:
        o, z = mem_pair(a, pes, pid, l_pac, ref)
        if o > 0:
            is_multi = any(any(r.secondary < 0 and r.score >= T for r in a[i][1:]) for i in range(2))
            if not is_multi:
                extra = 0
                if o > a[0][0].score + a[1][0].score - PEN_UNPAIRED:
                    extra |= 2
                else:
                    z = (0, 0)
                pick = [a[0][z[0]], a[1][z[1]]]
                out = []
                for i in range(2):
                    me = pick[i]
                    _, ts, _ = ref.locate(hs[i][me.k]["t_start"], hs[i][me.k]["t_end"])
                    flag, rnext, pnext = _mate_fields((0x40 << i) | extra | (0x10 if me.rev else 0),
                                                      ref.names[me.rid], ts + 1, me.rev, mate_of(1 - i, pick[1 - i]))
                    out.append(_record(ref, name, seqs[i], hs[i][me.k], me, flag, False, rnext, pnext))
                return out
    # no pairing: every record of each end (mem_reg2sam); the mate is the other end's top region
    top = [r[0] if r and r[0].score >= T else None for r in a]
    extra = 0
    if top[0] is not None and top[1] is not None and top[0].rid == top[1].rid:
        d, dist = infer_dir(l_pac, a[0][0].rb, a[1][0].rb)
        if not pes[d].failed and pes[d].low <= dist <= pes[d].high:
            extra |= 2
    out = []
    for i in range(2):
        out += se_records(ref, name, seqs[i], hs[i], None, None, T, extra_flag=(0x40 << i) | extra,
                          mate=mate_of(1 - i, top[1 - i]), regs=a[i])
    return out
