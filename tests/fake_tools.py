"""Deterministic stand-ins for the external tools the reference shells out to (BLAT, bedtools)
-- TEST INFRASTRUCTURE ONLY.

bwa, BLAT, samtools and bedtools are absent here (SURVEY.md §8 c), so the parity of the
consumer stages is pinned with synthetic tool outputs:

* tests/golden/make_fixtures.py intercepts the reference's `os.system` calls, reads the
  query/target files the reference wrote, and writes these functions' outputs where the
  tool would have written;
* the tests feed the same functions to the host restatement through its `place` /
  `getfasta` / `intersect` callbacks.

Every output is a pure function of its inputs (seeded by CRC32), so both sides see
identical records. The outputs mimic the tools' formats and the fields the reference reads.
They are NOT the tools' algorithms: placement parity with BLAT itself is unpinned.
"""
import random
import zlib

PSL_HEADER = ["psLayout version 3\n", "\n",
              "match\tmis- \trep. \tN's\tQ gap\tQ gap\tT gap\tT gap\tstrand\tQ        \tQ   \tQ    \tQ  \tT        "
              "\tT   \tT    \tT  \tblock\tblockSizes \tqStarts\t tStarts\n",
              "-" * 160 + "\n"]


def _rng(*key):
    return random.Random(zlib.crc32("|".join(map(str, key)).encode()))


def read_fasta_text(text):
    recs, name, buf = [], None, []
    for line in text.splitlines():
        if line.startswith(">"):
            if name is not None:
                recs.append((name, "".join(buf)))
            name, buf = line[1:].strip(), []
        elif line.strip():
            buf.append(line.strip())
    if name is not None:
        recs.append((name, "".join(buf)))
    return recs


def fasta_text(recs):
    return "".join(f">{n}\n{s}\n" for n, s in recs)


def _psl(matches, strand, qname, qsize, qs, qe, tname, tsize, ts, te):
    f = [str(matches), "0", "0", "0", "0", "0", "0", "0", strand, qname, str(qsize), str(qs), str(qe), tname,
         str(tsize), str(ts), str(te), "1", f"{max(qe - qs, 1)},", f"{qs},", f"{ts},"]
    return "\t".join(f) + "\n"


def blat(targets, queries, preset):
    """PSL placements of every query on the targets: 0-4 hits per query, with coordinates that
    exercise the consumers' edge windows (query ends, exon edges +-11, 0.9*qSize scores)."""
    out = list(PSL_HEADER)
    if not targets:
        return out
    for qname, qseq in queries:
        L = len(qseq)
        r = _rng("blat", preset, qname, qseq, len(targets))
        for _ in range(r.choice([0, 1, 1, 2, 2, 3, 4])):
            tname, tseq = targets[r.randrange(len(targets))]
            T = max(tseq if isinstance(tseq, int) else len(tseq), 1)
            kind = r.random()
            if kind < 0.25:
                qs, qe = 0, max(1, L - r.choice([0, 0, 0, 2, 6, 12]))
            elif kind < 0.45:
                qs, qe = r.choice([0, 1, 3, 5, 7, 12]), L
            elif kind < 0.65:
                qs, qe = r.choice([0, 0, 1, 2]), r.randint(L // 4, max(L // 4, 3 * L // 4))
            elif kind < 0.85:
                qs, qe = r.randint(L // 4, max(L // 4, 3 * L // 4)), L - r.choice([0, 0, 1])
            elif kind < 0.9:
                qs, qe = r.randint(0, max(0, L // 2)), L
            else:
                qs, qe = r.randint(0, max(0, L - 1)), r.randint(0, max(0, L))
                qs, qe = min(qs, qe), max(qs, qe)
            span = max(qe - qs, 1)
            ts = r.randint(0, max(0, T - span))
            te = ts + span + (r.randint(0, 400) if r.random() < 0.05 else 0)
            matches = span - (r.randint(0, max(1, span // 5)) if r.random() < 0.4 else 0)
            out.append(_psl(matches, r.choice("+-"), qname, L, qs, qe, tname, T, ts, te))
    return out


def genome_seq(chrom, start, end):
    """Synthetic reference bases for [start, end) (bedtools getfasta stand-in)."""
    r = _rng("genome", chrom, start // 1000)
    return "".join(r.choice("ACGT") for _ in range(max(0, end - start)))


def getfasta(bed_rows):
    """`bedtools getfasta -name` of (chrom, start, end, name) rows -> [(name::chrom:start-end, seq)]."""
    return [(f"{name}::{chrom}:{start}-{end}", genome_seq(chrom, start, end)) for chrom, start, end, name in bed_rows]


def intersect_wa(a_rows, b_rows):
    """`bedtools intersect -a A -b B -wa`: each A row once per overlapping B row (A order)."""
    out = []
    for a in a_rows:
        for b in b_rows:
            if a[0] == b[0] and int(a[1]) < int(b[2]) and int(b[1]) < int(a[2]):
                out.append(a)
    return out
