"""A small synthetic fusion sample for end-to-end pipeline tests (TEST INFRASTRUCTURE ONLY).

It builds:

- a genome (4 contigs) and a GTF (gene/transcript/exon rows, GENCODE-style attributes);
- an anchor gene BCRX on chr1 and a partner ABLX on chr2, plus background genes;
- paired FASTQs (2x100) from three sources:
  - the BCRX-ABLX fusion transcript (exons 1-3 of BCRX joined to exons 3-5 of ABLX);
  - the BCRX transcript;
  - background transcripts and intergenic sequence.

The truth is the junction in anchor-transcript coordinates (the end of BCRX exon 3) and the
partner genome position (the start of ABLX exon 3).
"""
import gzip
import os

import numpy as np

COMP = str.maketrans("ACGT", "TGCA")


def rc(s):
    return s.translate(COMP)[::-1]


def make_world(folder, seed=2024, n_fusion=400, n_anchor=300, n_background=1500, read_len=100):
    rng = np.random.default_rng(seed)
    bases = np.array(list("ACGT"))
    genome = [(f"chr{k}", "".join(rng.choice(bases, 60000))) for k in range(1, 5)]
    gseq = dict(genome)
    genes = []

    def add_gene(gid, name, chrom, start, n_exons):
        exons, p = [], start
        for _ in range(n_exons):
            ln = int(rng.integers(120, 260))
            exons.append((p, p + ln - 1))          # 1-based closed
            p += ln + int(rng.integers(600, 2500))
        genes.append((gid, name, chrom, exons))
        return exons

    bcr = add_gene("ENSG00000186716.21", "BCRX", "chr1", 5000, 6)
    abl = add_gene("ENSG00000097007.19", "ABLX", "chr2", 8000, 5)
    for k in range(8):
        add_gene(f"ENSG0000090{k:04d}.1", f"BG{k}", f"chr{1 + k % 4}", 30000 + 2000 * (k // 4), 3)

    def tx(exons, chrom):
        return "".join(gseq[chrom][s - 1:e] for s, e in exons)

    anchor = tx(bcr, "chr1")
    fusion = tx(bcr[:3], "chr1") + tx(abl[2:], "chr2")
    junction = sum(e - s + 1 for s, e in bcr[:3])
    gtf = ["##description: synthetic fusion world\n"]
    for gid, name, chrom, exons in genes:
        attrs = f'gene_id "{gid}"; gene_type "protein_coding"; gene_name "{name}"; level 2;'
        gtf.append("\t".join([chrom, "SYN", "gene", str(exons[0][0]), str(exons[-1][1]), ".", "+", ".", attrs]) + "\n")
        tattrs = f'gene_id "{gid}"; transcript_id "{gid}-T"; transcript_type "protein_coding"; gene_name "{name}";'
        gtf.append("\t".join([chrom, "SYN", "transcript", str(exons[0][0]), str(exons[-1][1]), ".", "+", ".",
                              tattrs]) + "\n")
        for k, (s, e) in enumerate(exons):
            gtf.append("\t".join([chrom, "SYN", "exon", str(s), str(e), ".", "+", ".",
                                  tattrs + f" exon_number {k + 1};"]) + "\n")

    def noisy(s):
        b = np.frombuffer(s.encode(), dtype=np.uint8).copy()
        m = rng.random(len(b)) < 0.005
        b[m] = np.frombuffer(rng.choice(bases, int(m.sum())).astype("S1"), dtype=np.uint8)
        return b.tobytes().decode()

    pairs = []

    def frag_pairs(src, n, tag, around=None):
        for i in range(n):
            F = int(rng.integers(220, 320))
            if around is not None:
                lo = max(0, around - F + 20)
                hi = min(len(src) - F, around - 20)
                s = int(rng.integers(lo, max(lo + 1, hi)))
            else:
                s = int(rng.integers(0, len(src) - F))
            frag = src[s:s + F]
            pairs.append((f"{tag}_{i}", noisy(frag[:read_len]), noisy(rc(frag[-read_len:]))))

    frag_pairs(fusion, n_fusion, "fus", around=junction)
    frag_pairs(anchor, n_anchor, "bcr")
    bg_src = [tx(ex, ch) for _, _, ch, ex in genes[2:]] + [gseq["chr3"][40000:52000], gseq["chr4"][5000:20000]]
    for i in range(n_background):
        src = bg_src[int(rng.integers(len(bg_src)))]
        frag_pairs(src, 1, f"bg{i}")
    order = rng.permutation(len(pairs))
    os.makedirs(folder, exist_ok=True)
    paths = {k: os.path.join(folder, v) for k, v in dict(
        fq1="s_1.fastq.gz", fq2="s_2.fastq.gz", genome="genome.fa", gtf="ann.gtf", anchor="anchor.fa").items()}
    with gzip.open(paths["fq1"], "wt") as f1, gzip.open(paths["fq2"], "wt") as f2:
        for k in order:
            name, r1, r2 = pairs[k]
            f1.write(f"@{name}/1\n{r1}\n+\n{'I' * len(r1)}\n")
            f2.write(f"@{name}/2\n{r2}\n+\n{'I' * len(r2)}\n")
    with open(paths["genome"], "w") as fh:
        for name, seq in genome:
            fh.write(f">{name}\n")
            for i in range(0, len(seq), 80):
                fh.write(seq[i:i + 80] + "\n")
    with open(paths["gtf"], "w") as fh:
        fh.writelines(gtf)
    with open(paths["anchor"], "w") as fh:
        fh.write(">NM_000000.1 BCRX transcript variant 1 mRNA\n")
        for i in range(0, len(anchor), 70):
            fh.write(anchor[i:i + 70] + "\n")
    truth = dict(anchor_junction=junction, partner_chrom="chr2", partner_pos=abl[2][0], anchor="BCRX",
                 partner="ABLX")
    return paths, truth
