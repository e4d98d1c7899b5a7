"""configs[0] end to end: the reference's bundled test set (tests/golden/test_sample_{1,2}.fastq.gz,
11,258 pairs x 101 bp, and target_gene.fasta, BCR NM_004327.4) through the whole pipeline
(Anchored_Fusion.py:181-227: S2 -> S3 -> S4/S5/S6 -> clustering -> S7/S8 -> Final_fusion) on the
C1 mini-genome + GTF built from the same data (tests/golden/make_c1_fixture.py: BCR and ABL1 as
exons of the transcript the reads were simulated from, EU216071.1).

CPU: the oracle backends (tests/oracle_backends.py) report the BCR-ABL1 fusion at the anchor's
3235 with the partner at ABL1 exon 2, and the anchor-side breakpoints (splitreads, fn:771-952)
hold 3235 (MS), 1848 (MS) and 2568 (SM) -- the three junctions the reads carry.
GPU: the product path writes the same two tables byte for byte and the same breakpoints."""
import os

import pytest

import afpkg  # noqa: F401
from anchored_fusion_amd import pipeline, splitreads

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
PATHS = dict(anchor=os.path.join(GOLD, "target_gene.fasta"), fq1=os.path.join(GOLD, "test_sample_1.fastq.gz"),
             fq2=os.path.join(GOLD, "test_sample_2.fastq.gz"), genome=os.path.join(GOLD, "c1", "c1_genome.fa"),
             gtf=os.path.join(GOLD, "c1", "c1_genes.gtf"))
TABLES = ("BCR_fusion_predictions.txt", "BCR_fusion_predictions_abridged.txt")
ABL1_EXON2 = 32315  # chr9, 1-based (make_c1_fixture.py prints it)


def _capture_breakpoints(monkeypatch):
    seen = []
    real = splitreads.cluster_split_reads

    def wrapped(sam_lines):
        bps = real(sam_lines)
        seen.append([(b.breakpoint, b.type_, b.cnt) for b in bps])
        return bps
    monkeypatch.setattr(splitreads, "cluster_split_reads", wrapped)
    return seen


def _run_oracle(out):
    from oracle_backends import OracleAligner, oracle_searches
    genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(PATHS["genome"])]
    pipeline.run(PATHS["anchor"], PATHS["fq1"], PATHS["fq2"], PATHS["genome"], PATHS["gtf"], out,
                 searches=oracle_searches(genome), aligner_factory=OracleAligner, log=lambda *_: None)


def _check(out, seen):
    assert len(seen) == 1
    kinds = {(bp, t) for bp, t, _ in seen[0]}
    for want in ((3235, "MS"), (1848, "MS"), (2568, "SM")):
        assert want in kinds, (want, sorted(seen[0], key=lambda x: -x[2])[:10])
    rows = [ln.rstrip("\n").split("\t") for ln in open(os.path.join(out, "BCR_fusion", TABLES[1]))]
    hit = [r for r in rows[1:] if "ABL1" in r[0]]
    assert hit, rows
    assert hit[0][2].split(":")[1] == "3235", hit[0]
    chrom, pos = hit[0][4].split(":")
    assert chrom == "chr9" and abs(int(pos) - ABL1_EXON2) <= 1, hit[0]
    return hit


def test_c1_oracle_backends_call_bcr_abl1(tmp_path, monkeypatch):
    seen = _capture_breakpoints(monkeypatch)
    out = str(tmp_path / "cpu")
    _run_oracle(out)
    _check(out, seen)


@pytest.mark.gpu
def test_c1_gpu_tables_equal_oracle(tmp_path, monkeypatch):
    """The product path on the GPU and the oracle backends: byte-identical tables, the same
    anchor-side breakpoints (with their read counts)."""
    seen = _capture_breakpoints(monkeypatch)
    gpu, cpu = str(tmp_path / "gpu"), str(tmp_path / "cpu")
    pipeline.run(PATHS["anchor"], PATHS["fq1"], PATHS["fq2"], PATHS["genome"], PATHS["gtf"], gpu, log=lambda *_: None)
    _run_oracle(cpu)
    assert len(seen) == 2 and seen[0] == seen[1]
    for t in TABLES:
        a = open(os.path.join(gpu, "BCR_fusion", t)).read()
        b = open(os.path.join(cpu, "BCR_fusion", t)).read()
        assert a == b, t
    _check(gpu, seen[:1])
