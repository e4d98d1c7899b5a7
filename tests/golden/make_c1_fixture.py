"""configs[0] (BASELINE.json: the bundled test/ FASTQ pair + target_gene.fasta) needs a genome and a
GTF for S4-S8 (SURVEY.md §8 d, C1: "synthetic mini-genome + GTF fixture ... not bundled in the
reference").  This script builds one from the reference's own test data (TEST INFRASTRUCTURE;
deterministic; run once, outputs committed under tests/golden/c1/):

1. The BCR-ABL1 transcript the bundled reads were simulated from.  Their names are wgsim's
   (`EU216071.1_<start>_<end>_...`: 1,702 of the 11,258 pairs come from GenBank EU216071.1, the
   rest from five other fusion transcripts).  Each pair's two reads sit at the fragment's ends,
   one forward and one reverse-complemented; the orientation of each pair is chosen by agreement
   with the consensus of the pairs placed so far (seeded by 20-mers of the anchor), iterated until
   no pair changes, and the per-position majority base is the transcript (5,369 of its 5,376 bases
   covered).  Against target_gene.fasta (BCR, NM_004327.4) it is anchor[452:1848] +
   anchor[2571:3235] + 3,311 bases that are not BCR (ABL1 from its exon a2): the junctions the
   reads show at anchor 1848 (MS), 2568 (SM; 3 nt of microhomology) and 3235 (MS).
2. A mini-genome: chr22 holds BCR as 11 exons of the anchor (exon ends at 1848, 2571 and 3235
   among them) with random introns, chr9 holds ABL1 (a random exon 1, then the transcript's
   non-BCR part as 7 exons), chr1 / chr5 random background with one gene each; seeded random
   bases, 30 kb flanks.
3. A GENCODE-style GTF of the four genes (gene / transcript / exon rows, transcript_type).

    python tests/golden/make_c1_fixture.py       -> tests/golden/c1/{c1_genome.fa, c1_genes.gtf, c1_transcript.txt}
"""
import gzip
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "c1")
COMP = str.maketrans("ACGTN", "TGCAN")
IDX = {c: i for i, c in enumerate("ACGT")}


def rc(s):
    return s.translate(COMP)[::-1]


def read_fq(path):
    out = []
    with gzip.open(path, "rt") as f:
        while True:
            h = f.readline()
            if not h:
                return out
            s = f.readline().strip()
            f.readline()
            f.readline()
            out.append((h.strip()[1:], s))


def anchor_seq():
    with open(os.path.join(HERE, "target_gene.fasta")) as f:
        return "".join(ln.strip() for ln in f if not ln.startswith(">"))


def reconstruct(anchor):
    r1 = read_fq(os.path.join(HERE, "test_sample_1.fastq.gz"))
    r2 = read_fq(os.path.join(HERE, "test_sample_2.fastq.gz"))
    pairs = []
    for (h, s1), (_, s2) in zip(r1, r2):
        if h.startswith("EU216071.1_"):
            f = h.split("_")
            pairs.append((int(f[1]) - 1, int(f[2]), s1, s2))
    L = max(en for _, en, _, _ in pairs) + 5
    akm = {anchor[i:i + 20] for i in range(len(anchor) - 19)}

    def hits(s):
        return sum(s[i:i + 20] in akm for i in range(0, len(s) - 20, 10))

    assign = []
    for st, en, s1, s2 in pairs:
        a, b = hits(s1) + hits(rc(s2)), hits(rc(s1)) + hits(s2)
        assign.append(0 if a > b else 1 if b > a else None)

    def consensus(assign):
        cnt = np.zeros((L, 4), np.int64)
        for (st, en, s1, s2), o in zip(pairs, assign):
            if o is None:
                continue
            fwd, rev = (s1, s2) if o == 0 else (s2, s1)
            for i, c in enumerate(fwd):
                if c in IDX:
                    cnt[st + i, IDX[c]] += 1
            rr = rc(rev)
            for i, c in enumerate(rr):
                if c in IDX:
                    cnt[en - len(rr) + i, IDX[c]] += 1
        return cnt

    for _ in range(100):
        cnt = consensus(assign)
        cons = "".join("ACGT"[int(np.argmax(c))] if c.sum() else "N" for c in cnt)
        new = []
        for st, en, s1, s2 in pairs:
            def agree(fwd, rev):
                rr = rc(rev)
                return (sum(x == y for x, y in zip(fwd, cons[st:st + len(fwd)])) +
                        sum(x == y for x, y in zip(rr, cons[en - len(rr):en])))
            a, b = agree(s1, s2), agree(s2, s1)
            new.append(0 if a > b else 1 if b > a else None)
        changed = sum(x != y for x, y in zip(new, assign))
        assign = new
        if changed == 0:
            break
    cnt = consensus(assign)
    return "".join("ACGT"[int(np.argmax(c))] if c.sum() else "N" for c in cnt)


def main():
    anchor = anchor_seq()
    cons = reconstruct(anchor)
    # the transcript's BCR part, as the reads show it
    def diff(a, b):
        return sum(x != y for x, y in zip(a, b))
    assert diff(cons[2:1396], anchor[454:1848]) <= 4 and diff(cons[1396:2060], anchor[2571:3235]) <= 4, "unexpected transcript"
    partner = cons[2060:5371]
    assert "N" not in partner
    rng = np.random.default_rng(20251015)

    def rand(n):
        return "".join(rng.choice(list("ACGT"), n))

    genome, genes = {}, []

    def build(chrom, pieces, flank=30000):
        """pieces: [(gene, exon seq) ...] laid out with random introns; returns exon coordinates."""
        seq = [rand(flank)]
        pos = flank
        coords = {}
        for gene, ex in pieces:
            if gene in coords:
                ln = int(rng.integers(800, 3000))
                seq.append(rand(ln))
                pos += ln
            coords.setdefault(gene, []).append((pos + 1, pos + len(ex)))  # 1-based closed
            seq.append(ex)
            pos += len(ex)
        seq.append(rand(flank))
        genome[chrom] = "".join(seq)
        return coords

    bcr_cuts = [0, 452, 1100, 1848, 2571, 2900, 3235, 3800, 4400, 5100, 5900, len(anchor)]
    bcr = build("chr22", [("BCR", anchor[a:b]) for a, b in zip(bcr_cuts, bcr_cuts[1:])])["BCR"]
    abl_cuts = [0, 174, 470, 650, 900, 1200, 1650, len(partner)]
    abl = build("chr9", [("ABL1", rand(280))] + [("ABL1", partner[a:b]) for a, b in zip(abl_cuts, abl_cuts[1:])])["ABL1"]
    bg1 = build("chr1", [("BGA", rand(int(rng.integers(150, 400)))) for _ in range(4)], flank=50000)["BGA"]
    bg5 = build("chr5", [("BGB", rand(int(rng.integers(150, 400)))) for _ in range(3)], flank=50000)["BGB"]
    genes = [("ENSG00000186716.21", "BCR", "chr22", bcr), ("ENSG00000097007.19", "ABL1", "chr9", abl),
             ("ENSG00000900001.1", "BGA", "chr1", bg1), ("ENSG00000900002.1", "BGB", "chr5", bg5)]
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "c1_genome.fa"), "w") as fh:
        for chrom in ("chr1", "chr5", "chr9", "chr22"):
            fh.write(f">{chrom}\n")
            s = genome[chrom]
            for i in range(0, len(s), 80):
                fh.write(s[i:i + 80] + "\n")
    with open(os.path.join(OUT, "c1_genes.gtf"), "w") as fh:
        fh.write("##description: C1 mini-genome (tests/golden/make_c1_fixture.py)\n")
        for gid, name, chrom, exons in genes:
            attrs = f'gene_id "{gid}"; gene_type "protein_coding"; gene_name "{name}"; level 2;'
            fh.write("\t".join([chrom, "SYN", "gene", str(exons[0][0]), str(exons[-1][1]), ".", "+", ".", attrs]) + "\n")
            t = f'gene_id "{gid}"; transcript_id "{gid}-T"; transcript_type "protein_coding"; gene_name "{name}";'
            fh.write("\t".join([chrom, "SYN", "transcript", str(exons[0][0]), str(exons[-1][1]), ".", "+", ".", t]) + "\n")
            for k, (s, e) in enumerate(exons):
                fh.write("\t".join([chrom, "SYN", "exon", str(s), str(e), ".", "+", ".", t + f" exon_number {k + 1};"]) + "\n")
    with open(os.path.join(OUT, "c1_transcript.txt"), "w") as fh:
        fh.write(cons + "\n")
    # where the fusion junction lies on the genome: ABL1 exon 2's first base (1-based)
    print("BCR exons", bcr)
    print("ABL1 exon 2 starts at chr9:", abl[1][0])


if __name__ == "__main__":
    main()
