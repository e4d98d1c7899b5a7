"""Replays the a9-a14 partner chain of tests/golden/consumers.json through the host
restatement (TEST INFRASTRUCTURE ONLY).

Run under PYTHONHASHSEED=0, as the fixture generator was. The reference splits spanning reads
by `list(set(...))` order (functions.py:1320-1324), so the exact lists depend on string
hashing. test_consumers.py::test_partner_chain starts this script in a subprocess. It exits 0
on success, 1 on the first mismatch.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import afpkg  # noqa: E402,F401
import fake_tools  # noqa: E402
from anchored_fusion_amd import annotation, blocks, partner, report, splitreads  # noqa: E402


def sanitize(blocks_chr):
    for c in list(blocks_chr):
        blocks_chr[c] = [b for b in blocks_chr[c] if isinstance(b.start, int) and isinstance(b.end, int)]


def main():
    with open(os.path.join(HERE, "golden", "consumers.json")) as fh:
        fx = json.load(fh)
    index = annotation.ExonIndex.from_lines(fx["gtf"])
    homo = fx["homo_genes"]
    P = fx["partner"]
    genome = [tuple(g) for g in P["genome"]]
    small = [tuple(g) for g in P["small_genome"]]
    anchor = tuple(P["anchor"])

    def check(what, got, want):
        if got != want:
            print("MISMATCH", what)
            print(" got ", json.dumps(got)[:2000])
            print(" want", json.dumps(want)[:2000])
            sys.exit(1)

    for anc, rows in P["homologs"]:
        got = partner.homolog_genes(fx["gtf"], small, [tuple(anc)], fake_tools.blat)
        check("homologs", ["\t".join(r) + "\n" for r in got], rows)

    for t, trial in enumerate(P["trials"]):
        calls = []

        def place(targets, queries, preset):
            calls.append([preset, [list(q) for q in queries]])
            return fake_tools.blat(targets, queries, preset)

        bc = blocks.spanning_blocks(trial["spanning"], index, homo)
        sanitize(bc)
        recs = partner.candidate_targets(bc, fake_tools.getfasta, place, [anchor])
        check(f"{t} candidate records", [list(r) for r in recs], trial["candidate_records"])
        check(f"{t} blocks after a10", {c: [[b.chrom, b.start, b.end, b.count] for b in bl] for c, bl in bc.items()},
              trial["blocks_after_a10"])
        bps = splitreads.cluster_split_reads(trial["split"])
        good = partner.anchored_split_placement(recs, bc, bps, index, place, [anchor])
        check(f"{t} a9 good", sorted(good), trial["a9"]["good"])
        check(f"{t} a9 breakpoints", [list(b.as_tuple()) + [[list(o) for o in b.other_breakpoints]] for b in bps],
              trial["a9"]["breakpoints"])
        check(f"{t} a9 anchored", {c: [sorted(b.anchored_split_breakpoints) for b in bl] for c, bl in bc.items()},
              trial["a9"]["anchored"])
        cands, cnt_max = partner.candidate_genes(good, bps, bc, place, genome)
        got = [dict(type=c.type_, pos=[list(p) for p in c.pos], left=c.left_seq(), right=c.right_seq(),
                    mid=c.mid_seq(), l=[c.l_left, c.l_mid, c.l_right], spanning=list(c.spanning_reads),
                    split=list(c.split_reads)) for c in cands]
        check(f"{t} a11", dict(candidates=got, cnt_max=cnt_max, error=None), trial["a11"])
        check(f"{t} tool calls", calls, trial["blat_calls"])
        ab, full = report.prediction_rows(cands, "BCR", index, [], cnt_max, True)
        check(f"{t} abridged", [r + "\n" for r in ab], trial["final"]["abridged"][1:])
        check(f"{t} full", [r + "\n" for r in full], trial["final"]["full"][1:])
    print("partner chain OK:", len(P["trials"]), "trials")


if __name__ == "__main__":
    main()
