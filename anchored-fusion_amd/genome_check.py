"""Genome check of anchored split reads.

Restates the two ends of `del_too_many_reads` (functions.py:705-768) around its `bwa mem`
call against the genome (fn:716).

* `split_read_fasta` selects the anchored primary records whose CIGAR normalises to exactly
  two ops. It names each one `QNAME$RNAME$POS$CIGAR` and keeps the SEQ as stored (fn:710-715).
* `filter_genome_hits` walks the genome SAM for those queries. Records are grouped by
  consecutive query name, and a query is dropped (bad) when either of these holds:
  - a genome record aligns it as a single op (the whole read lies elsewhere in the genome);
  - a genome M straddles an anchored M's end by more than 20 % of the anchored M's length on
    both sides (fn:749-756).
  Reverse records (0x10) are reverse-complemented and their ops reversed first. The first H
  of a CIGAR is read as S.
  Every surviving query becomes one pseudo-SAM line: `QNAME 0 RNAME POS 60 CIGAR = 1111 0
  SEQ A` (fn:735, 760).

As in the reference, the last group is only flushed when the file's last line is a record.
"""
from .cigar import normalize, revcomp


def split_read_fasta(anchored_sam_lines):
    out = []
    for line in anchored_sam_lines:
        f = line.split("\t")
        ops, _ = normalize(f[5], f[9])
        if len(ops) == 2:
            out.append(("$".join([f[0], f[2], f[3], f[5]]), f[9]))
    return out


def _is_rev(flag):
    return flag > 15 and (flag >> 4) & 1 == 1


def _emit(name, seq):
    q, rname, pos, cigar = name.split("$")[:4]
    return f"{q}\t0\t{rname}\t{pos}\t60\t{cigar}\t=\t1111\t0\t{seq}\tA\n"


def filter_genome_hits(genome_sam_lines):
    out = []
    cur, cur_seq, bad = "", "", 0
    last = len(genome_sam_lines) - 1
    for n, line in enumerate(genome_sam_lines):
        if line.startswith("@"):
            continue
        f = line.split("\t")
        flag = int(f[1])
        rev = _is_rev(flag)
        if rev:
            f[9] = revcomp(f[9])
        if f[0] != cur:
            if bad == 0 and cur != "":
                out.append(_emit(cur, cur_seq))
            cur, bad, cur_seq = f[0], 0, f[9]
        if bad == 0:
            cig = f[5]
            h = cig.find("H")
            if h > -1:
                cig = cig[:h] + "S" + cig[h + 1:]
            now, _ = normalize(cig, f[9])
            before, _ = normalize(f[0].split("$")[3], f[9])
            if rev:
                now = now[::-1]
                run = 0
                for op in now:
                    run += op[1]
                    op[0] = run
            if len(now) == 1:
                bad = 1
            elif len(now) >= 2:
                for a in before:
                    if a[2] != "M":
                        continue
                    lo, hi = a[0] - a[1] * 0.2, a[0] + a[1] * 0.2
                    if any(g[2] == "M" and g[0] - g[1] < lo and g[0] > hi for g in now):
                        bad = 1
        if n == last and bad == 0 and cur != "":
            out.append(_emit(cur, cur_seq))
    return out
