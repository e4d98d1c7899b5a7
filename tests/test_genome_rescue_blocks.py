"""S4's mate rescue decides Find_blocks' output (functions.py:376-496 over `bwa mem -M genome tmp1
tmp2`, AF:188): the genome engine (oracle/bwa_pe.c FM mode, the contract the GPU's
csrc/bwa_genome.hip meets bit-exactly) with bwa's mem_matesw places a mate that has no exact
19-mer (a mismatch every 12 bases) from its partner's position and the chunk's insert-size
statistics; that mate lies in a partner gene 2.5 kb downstream of the anchor gene, so the pair
becomes spanning evidence and `spanning_blocks` opens a block on the partner gene.  With rescue
off (max_matesw = 0) the mate stays unmapped and no block appears -- the crafted case the
single-seed engine of round 2 (no rescue on the genome) got wrong.  The GPU side:
tests/test_gpu_genome.py compares the kernel's records with this engine's on the same pairs."""
import numpy as np

import afpkg  # noqa: F401
import oracle
from anchored_fusion_amd import blocks, genome
from anchored_fusion_amd.annotation import ExonIndex

ACGT = np.frombuffer(b"ACGT", np.uint8)
L, INS = 150, 2500
ANCHOR_EXON = (40_000, 40_600)     # anchor gene exon on chrA (0-based half-open)
PARTNER_EXON = (42_200, 42_900)    # partner gene exon 2.2 kb downstream


def _rc(s):
    return np.frombuffer(s[::-1].tobytes().translate(bytes.maketrans(b"ACGT", b"TGCA")), np.uint8)


def crafted():
    rng = np.random.default_rng(11)
    chrA = ACGT[rng.integers(0, 4, 200_000)]
    chrB = ACGT[rng.integers(0, 4, 150_000)]
    contigs = [("chrA", chrA.tobytes().decode()), ("chrB", chrB.tobytes().decode())]
    pairs = []
    # proper FR pairs with a 2.5 kb insert (the chunk's insert-size statistics)
    for _ in range(300):
        g = chrA if rng.random() < 0.6 else chrB
        a = int(rng.integers(60_000 if g is chrA else 0, len(g) - INS - 10))
        ins = INS + int(rng.integers(-40, 41))
        frag = g[a:a + ins]
        pairs.append((frag[:L].copy(), _rc(frag[-L:])))
    # the probe: mate 1 in the anchor exon, mate 2 in the partner exon, a mismatch every 12 bases
    a = ANCHOR_EXON[0] + 100
    frag = chrA[a:a + INS]
    m2 = _rc(frag[-L:]).copy()
    for k in range(6, L, 12):
        m2[k] = ord("A") if m2[k] != ord("A") else ord("G")
    pairs.append((frag[:L].copy(), m2))
    reads = np.stack([r for p in pairs for r in p])
    gtf = []
    for gid, name, (s, e) in (("ENSG00000000001.1", "ANCH", ANCHOR_EXON), ("ENSG00000000002.1", "PART", PARTNER_EXON)):
        attrs = f'gene_id "{gid}"; gene_type "protein_coding"; gene_name "{name}"; level 2;'
        ta = f'gene_id "{gid}"; transcript_id "{gid}-T"; transcript_type "protein_coding"; gene_name "{name}";'
        gtf.append("\t".join(["chrA", "SYN", "gene", str(s + 1), str(e), ".", "+", ".", attrs]) + "\n")
        gtf.append("\t".join(["chrA", "SYN", "transcript", str(s + 1), str(e), ".", "+", ".", ta]) + "\n")
        gtf.append("\t".join(["chrA", "SYN", "exon", str(s + 1), str(e), ".", "+", ".", ta + " exon_number 1;"]) + "\n")
    return contigs, reads, ExonIndex.from_lines(gtf)


def _blocks(og, reads, index, max_matesw):
    pe = oracle.default_pe()
    pe.max_matesw = max_matesw
    recs, nrec = og.align_pe(reads, np.full(len(reads), L, np.int32), pe=pe, pair_base=0, threads=4)
    names = [f"p{k}" for k in range(len(reads) // 2)]
    lines = []
    for k, nm in enumerate(names):
        for m in (0, 1):
            r = 2 * k + m
            lines += genome.sam_lines(og.names, nm, reads[r].tobytes().decode(), recs[r], nrec[r])
    probe = recs[len(reads) - 1, 0]
    return blocks.spanning_blocks(lines, index, ["ENSG00000000001.1"]), probe


def test_mate_rescue_opens_the_partner_block():
    contigs, reads, index = crafted()
    og = oracle.OracleGenome(contigs)
    with_rescue, probe = _blocks(og, reads, index, 50)
    assert not probe["flag"] & 4 and probe["rid"] == 0 and abs(int(probe["pos"]) - (ANCHOR_EXON[0] + 100 + INS - L)) < 5
    got = {c: [(b.start, b.end, b.gene[1], b.count) for b in bl] for c, bl in with_rescue.items()}
    assert list(got) == ["chrA"] and len(got["chrA"]) == 1 and got["chrA"][0][2] == "PART" and got["chrA"][0][3] == 1
    without, probe0 = _blocks(og, reads, index, 0)
    assert probe0["flag"] & 4
    assert without == {}
