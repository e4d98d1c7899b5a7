"""Partner placement stages around the tail searches.

These restate the consumer logic of the reference's BLAT/bedtools stages. The searches are
callbacks, so the same logic runs against the GPU tail placement (`anchored_fusion_amd.place`)
in production and against deterministic stand-ins in the parity tests:

    place(targets, queries, preset) -> PSL lines   (targets/queries: [(name, seq)])
    getfasta(bed_rows) -> [(name::chrom:start-end, seq)]

| function | reference | what it does |
|---|---|---|
| `homolog_genes` | Find_homo_genes fn:336-373 | anchor vs genome (preset "homologs") ∩ GTF gene rows |
| `candidate_targets` | Build_candidate_fasta fn:955-991 | blocks ±100 nt; drop blocks the anchor hits ("candidate_homolog") |
| `anchored_split_placement` | Find_Anchored_split fn:994-1145 | clipped halves vs candidate blocks, exon-edge snapping + re-search, anchored half vs anchor |
| `candidate_genes` | Find_candidate_genes fn:1148-1329 | shortest placements, consensus candidates, genome validation ("genome_validate") |

The quirks are kept: the `i == len(lines) - 1` early stop of the validation loop, the
dedup test that compares a coordinate with a chromosome name, the spanning-read rebalance
that depends on `list(set(...))` order, and the `e + add_length - l` snapping shifts.
"""
import re

from .report import Candidate

_PSL = re.compile(r"^\d+\s")

PRESETS = {
    "homologs": "-stepSize=3 -repMatch=10000 -minScore=50 -minIdentity=80",
    "candidate_homolog": "-stepSize=3 -minScore=20 -minMatch=2 -minIdentity=0",
    "anchored_split": "-stepSize=3 -minScore=12 -minMatch=2 -minIdentity=90",
    "genome_validate": "-stepSize=3 -minScore=20 -minMatch=3 -minIdentity=90",
    "split_tail": "-minScore=20",
}


def psl_rows(lines, pattern=_PSL):
    return [ln.split("\t") for ln in lines if pattern.match(ln)]


# ---- a13 -------------------------------------------------------------------------------------
_GENE_RE = re.compile(r'gene_id\s+"(ENSG\d+\S+)";\s+.+gene_name\s+"(\S+)";\s+')


def gtf_gene_rows(gtf_lines):
    out = []
    for line in gtf_lines:
        if line.startswith("##"):
            continue
        f = line.split("\t")
        if f[2] != "gene":
            continue
        m = _GENE_RE.findall(f[8])
        if m:
            out.append([f[0], f[3], f[4], m[0][0], m[0][1], f[6]])
    return out


def intersect_wa(a_rows, b_rows):
    """bedtools intersect -a A -b B -wa: A rows in A order, once per overlapping B row."""
    out = []
    for a in a_rows:
        for b in b_rows:
            if a[0] == b[0] and int(a[1]) < int(b[2]) and int(b[1]) < int(a[2]):
                out.append(a)
    return out


def homolog_genes(gtf_lines, genome_targets, anchor_records, place, intersect=intersect_wa):
    """Rows of <G>_homo_genes.bed (chrom, start, end, gene_id, gene_name, strand)."""
    hits = [ln.split("\t") for ln in place(genome_targets, anchor_records, "homologs") if re.match(r"^\d+", ln)]
    bed = [[f[13], f[15], f[16], f[9], f[8]] for f in hits]
    return intersect(gtf_gene_rows(gtf_lines), bed)


# ---- a10 -------------------------------------------------------------------------------------
def candidate_targets(blocks_chr, getfasta, place, anchor_records):
    """Candidate partner sequences (the second getfasta of fn:986); blocks hit by the anchor
    are marked bad and removed from blocks_chr."""
    rows = []
    for blocks in blocks_chr.values():
        for i, b in enumerate(blocks):
            b.start -= 100
            b.end += 100
            rows.append((b.chrom, b.start, b.end, str(i)))
    first = getfasta(rows)
    for f in psl_rows(place(first, anchor_records, "candidate_homolog")):
        bid, rest = f[13].split("::", 1)
        blocks_chr[rest.split(":")[0]][int(bid)].bad = True
    rows = []
    for chrom in list(blocks_chr):
        kept = [b for b in blocks_chr[chrom] if b.bad is not True]
        blocks_chr[chrom][:] = kept
        rows.extend((b.chrom, b.start, b.end, str(i)) for i, b in enumerate(kept))
    return getfasta(rows)


# ---- a9 --------------------------------------------------------------------------------------
def _target_coords(tname):
    bid, rest = tname.split("::", 1)
    chrom, span = rest.split(":")[0], rest.split(":")[1]
    return int(bid), chrom, int(span.split("-")[0])


def anchored_split_placement(candidate_records, blocks_chr, breakpoints, index, place, anchor_records):
    """Set of breakpoint ids whose clipped half lands on a candidate block and whose anchored
    half lies on the anchor (>= 0.9 x length matches)."""
    queries = [(str(i), bp.seq_left if bp.type_ == "SM" else bp.seq_right) for i, bp in enumerate(breakpoints)]
    good = set()
    retry = []
    for f in psl_rows(place(candidate_records, queries, "anchored_split")):
        L, s, e = int(f[10]), int(f[11]), int(f[12])
        if s > 5 and e < L - 5:
            continue
        bid, chrom_y, base = _target_coords(f[13])
        ys, ye, strand = int(f[15]) + base + 1, int(f[16]) + base, f[8]
        bp = breakpoints[int(f[9])]
        qid = int(f[9])
        if bp.type_ == "SM":
            at = ye if strand == "+" else ys
            exon = index.find_exon(chrom_y, at, at)[0]
            if exon[0] == "":
                continue
            if strand == "+" and exon[4] - 11 < ye < exon[4] and e == L:
                retry.append((f"{qid}${exon[4] - ye}", bp.seq_left + bp.seq_right[:exon[4] - ye]))
                continue
            if strand != "+" and exon[3] < ys < exon[3] + 11 and e == L:
                retry.append((f"{qid}${ys - exon[3]}", bp.seq_left + bp.seq_right[:ys - exon[3]]))
                continue
            bp.Add_other_breakpoint(chrom_y, at, strand, s, L - e)
        else:
            at = ys if strand == "+" else ye
            exon = index.find_exon(chrom_y, at, at)[0]
            if exon[0] == "":
                continue
            if strand == "+" and exon[3] < ys < exon[3] + 11 and s == 0:
                retry.append((f"{qid}${ys - exon[3]}", bp.seq_left[exon[3] - ys:] + bp.seq_right))
                continue
            if strand != "+" and exon[4] - 11 < ye < exon[4] and s == 0:
                retry.append((f"{qid}${exon[4] - 1 - ye}", bp.seq_left[ye - exon[4]:] + bp.seq_right))
                continue
            bp.Add_other_breakpoint(chrom_y, at, strand, s, L - e)
        blocks_chr[chrom_y][bid].anchored_split_breakpoints.add(qid)
        good.add(qid)
    if retry:
        for f in psl_rows(place(candidate_records, retry, "anchored_split")):
            L, s, e = int(f[10]), int(f[11]), int(f[12])
            qid, add = (int(x) for x in f[9].split("$"))
            bid, chrom_y, base = _target_coords(f[13])
            ys, ye, strand = int(f[15]) + base + 1, int(f[16]) + base, f[8]
            bp = breakpoints[qid]
            if bp.type_ == "SM":
                if e > L - add:
                    sh = e + add - L
                    bp.breakpoint += sh
                    bp.seq_left += bp.seq_right[:sh]
                    bp.seq_right = bp.seq_right[sh:]
                bp.Add_other_breakpoint(chrom_y, ye if strand == "+" else ys, strand, s, L - e)
            else:
                if s < add:
                    bp.seq_right = bp.seq_left[s - add:] + bp.seq_right
                    bp.seq_left = bp.seq_left[:s - add]
                    bp.breakpoint -= add - s
                bp.Add_other_breakpoint(chrom_y, ys if strand == "+" else ye, strand, s, L - e)
            blocks_chr[chrom_y][bid].anchored_split_breakpoints.add(qid)
            good.add(qid)
    halves = []
    for qid in good:
        bp = breakpoints[qid]
        if bp.type_ == "SM":
            halves.append((str(qid), bp.seq_right))
        elif bp.type_ == "MS":
            halves.append((str(qid), bp.seq_left))
    final = set()
    for f in psl_rows(place(anchor_records, halves, "anchored_split")):
        if int(f[10]) * 0.9 <= int(f[0]):
            final.add(int(f[9]))
    return final


# ---- a11 -------------------------------------------------------------------------------------
def _agree(a, b):
    n = min(len(a), len(b))
    return sum(1 for x in range(n) if a[x] == b[x]) / n


def _similar(l1, r1, l2, r2, m1, m2, thr):
    """functions.py:1155-1180."""
    if not (l1 and l2 and r1 and r2):
        return False
    if m1 and m2:
        if _agree(m1, m2) < thr:
            return False
    elif (len(m1) > 3 and not m2) or (len(m2) > 3 and not m1):
        return False
    return _agree(l1[::-1], l2[::-1]) > thr and _agree(r1, r2) > thr


def _keep_shortest(breakpoints):
    for bp in breakpoints:
        best = 1000
        for ob in bp.other_breakpoints:
            best = min(best, ob[-1] + ob[-2])
        bp.other_breakpoints[:] = [ob for ob in bp.other_breakpoints if ob[-1] + ob[-2] == best]


def _validate(candidates, psl_lines):
    """Genome check of each candidate's left+mid+right (fn:1250-1290): a candidate is good when
    one placement covers the left half, another the right half, and none spans both."""
    good = []
    lines = psl_lines
    i, name = 0, -1
    L = M = R = 0
    while i < len(lines):
        if not _PSL.match(lines[i]):
            i += 1
            continue
        j, bad, state = 0, 0, 0
        if name != -1:
            c = candidates[name]
            L, M, R = c.l_left, c.l_mid, c.l_right
        while i + j <= len(lines):
            if i + j == len(lines):
                if name != -1 and bad == 0 and state == 3:
                    good.append(name)
                break
            f = lines[i + j].split("\t")
            q, s, e = int(f[9]), int(f[11]), int(f[12])
            if q != name:
                if name != -1 and bad == 0 and state == 3:
                    good.append(name)
                name = q
                break
            if s < L * 0.5 and e > L * 1.5 + M:
                bad = 1
            elif s <= L * 0.5 and L * 0.5 <= e <= L * 1.5:
                state = {0: 1, 2: 3}.get(state, state)
            elif L + M - R * 0.5 <= s <= L + M + R * 0.5 and L + M + R * 0.5 <= e:
                state = {0: 2, 1: 3}.get(state, state)
            j += 1
        i += j
        if i == len(lines) - 1:
            break
    return good


def candidate_genes(breakpoint_good, breakpoints, blocks_chr, place, genome_targets):
    """(candidates, cnt_max) as Find_candidate_genes returns them."""
    _keep_shortest(breakpoints)
    cands = []
    for blocks in blocks_chr.values():
        for block in blocks:
            for qid in block.anchored_split_breakpoints:
                bp = breakpoints[qid]
                if not bp.other_breakpoints or qid not in breakpoint_good:
                    continue
                for ob in bp.other_breakpoints:
                    if ob[0] != block.chrom:
                        continue
                    left, right, mid = bp.seq_left, bp.seq_right, ""
                    if bp.type_ == "SM":
                        left = left[ob[-2]:]
                        if ob[-1] != 0:
                            left, mid = left[:-ob[-1]], left[-ob[-1]:]
                    elif bp.type_ == "MS":
                        mid, right = right[:ob[-2]], right[ob[-2]:]
                        if ob[-1] != 0:
                            right = right[:-ob[-1]]
                    home = None
                    for c in reversed(cands[max(0, len(cands) - 200):]):
                        if c.type_ == bp.type_ and _similar(c.left_seq(), c.right_seq(), left, right, c.mid_seq(),
                                                            mid, 0.9):
                            home = c
                            break
                    if home is None:
                        home = Candidate(bp.type_)
                        cands.append(home)
                    home.add_reads(bp.breakpoint, ob, left, right, mid, bp.cnt, block.reads, bp.reads)
    good = []
    if cands:
        queries = [(str(i), c.left_seq() + c.mid_seq() + c.right_seq()) for i, c in enumerate(cands)]
        good = _validate(cands, place(genome_targets, queries, "genome_validate"))
    cnt_max = 0
    picked = []
    for i, c in enumerate(cands):
        if i in good:
            pos = c.find_max_pos()[0]
            picked.append((c, pos))
            cnt_max = max(cnt_max, pos[6])
    out, kept = [], []
    for c, pos in picked:
        # the reference compares pos[0] (a coordinate) with the kept ones' coordinate AND chromosome
        if any(pos[0] == q[0] and pos[0] == q[1] and pos[0] == q[2] for q in kept):
            continue
        kept.append(pos)
        out.append(c)
    for c in out:
        if len(c.spanning_reads) * 3 < len(c.split_reads) or len(c.split_reads) * 3 < len(c.spanning_reads):
            p = c.find_max_pos()[0]
            for c2 in out:
                p2 = c2.find_max_pos()[0]
                if abs(p2[0] - p[0]) < 100 and p[1] == p2[1] and (p[2] - p2[2]) < 100:
                    ratio = len(c.split_reads) / (len(c.split_reads) + len(c2.split_reads))
                    pool = list(set(c.spanning_reads + c2.spanning_reads))
                    cut = int(ratio * len(pool))
                    c.spanning_reads = pool[:cut]
                    c2.spanning_reads = pool[cut:]
    return out, cnt_max
