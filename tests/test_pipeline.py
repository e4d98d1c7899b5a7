"""End-to-end runs of the fusion pipeline (anchored_fusion_amd.pipeline) on a synthetic
fusion sample.

The CPU test swaps the GPU search services for the oracle (tests/oracle_backends.py). The
GPU test runs the product path. Both must report the planted BCRX-ABLX fusion, with its anchor
breakpoint within a few bases of the junction; and on the same world the GPU pipeline's
candidate tables must equal the oracle pipeline's byte for byte (the whole §8 a chain:
S2 records -> partitions -> genome/partner searches -> clustering -> Final_fusion).
"""
import os

import pytest

import afpkg  # noqa: F401
from anchored_fusion_amd import pipeline
from fusion_world import make_world


def _check(out_folder, truth):
    pred = os.path.join(out_folder, "BCRX_fusion", "BCRX_fusion_predictions_abridged.txt")
    full = os.path.join(out_folder, "BCRX_fusion", "BCRX_fusion_predictions.txt")
    assert os.path.exists(pred) and os.path.exists(full)
    rows = [ln.rstrip("\n").split("\t") for ln in open(pred)][1:]
    assert rows, "no fusion predicted"
    hit = [r for r in rows if "ABLX" in r[0]]
    assert hit, rows
    bp = int(hit[0][2].split(":")[1])
    assert abs(bp - truth["anchor_junction"]) <= 3, (bp, truth)
    assert hit[0][4].startswith("chr2:")
    return hit


def _run_oracle(paths, out):
    from oracle_backends import OracleAligner, oracle_searches
    genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
    searches = oracle_searches(genome)
    pipeline.run(paths["anchor"], paths["fq1"], paths["fq2"], paths["genome"], paths["gtf"], out,
                 searches=searches, aligner_factory=OracleAligner, log=lambda *_: None)


def test_pipeline_cpu_backends(tmp_path):
    paths, truth = make_world(str(tmp_path / "world"))
    out = str(tmp_path / "out")
    _run_oracle(paths, out)
    _check(out, truth)


TABLES = ("BCRX_fusion_predictions.txt", "BCRX_fusion_predictions_abridged.txt")


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_fusion", [(2024, 400), (7, 400), (99, 60), (5, 1200)])
def test_pipeline_gpu_tables_equal_oracle(tmp_path, seed, n_fusion):
    """GPU pipeline vs the CPU-oracle pipeline on the same world: identical TSVs."""
    paths, truth = make_world(str(tmp_path / "world"), seed=seed, n_fusion=n_fusion)
    gpu, cpu = str(tmp_path / "gpu"), str(tmp_path / "cpu")
    pipeline.run(paths["anchor"], paths["fq1"], paths["fq2"], paths["genome"], paths["gtf"], gpu,
                 log=lambda *_: None)
    _run_oracle(paths, cpu)
    for t in TABLES:
        a = open(os.path.join(gpu, "BCRX_fusion", t), "rb").read()
        b = open(os.path.join(cpu, "BCRX_fusion", t), "rb").read()
        assert a == b, (t, a[:2000], b[:2000])
    rows = [ln.split("\t") for ln in open(os.path.join(gpu, "BCRX_fusion", TABLES[1]))][1:]
    if n_fusion >= 400:  # at 60 fusion pairs too few split-read tails carry BLAT's two 11-mer tiles
        assert any("ABLX" in r[0] for r in rows)


@pytest.mark.gpu
def test_pipeline_gpu(tmp_path):
    paths, truth = make_world(str(tmp_path / "world"))
    out = str(tmp_path / "out")
    pipeline.run(paths["anchor"], paths["fq1"], paths["fq2"], paths["genome"], paths["gtf"], out)
    _check(out, truth)


@pytest.mark.gpu
def test_cli_gpu(tmp_path):
    import subprocess
    import sys
    paths, truth = make_world(str(tmp_path / "world"), seed=7)
    out = str(tmp_path / "cli_out")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "run_anchored_fusion.py"), "--file_anchored_cds",
                        paths["anchor"], "--fastq1", paths["fq1"], "--fastq2", paths["fq2"], "--file_ref_seq",
                        paths["genome"], "--file_ref_ann", paths["gtf"], "--out_folder", out,
                        "--not_filter_false_positive", "--thread", "4"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(out, truth)


def test_pipeline_filter_step_cpu_backends(tmp_path):
    """AF:212-225 wired: with a model file the candidates are scored (get_test_reads ->
    Test_model) and Final_fusion writes the Natural_score layout; a missing model file gives the
    unfiltered tables, as in the reference."""
    import torch
    from oracle_backends import OracleAligner, oracle_searches
    from anchored_fusion_amd import filter_model
    from anchored_fusion_amd.annotation import ExonIndex
    paths, truth = make_world(str(tmp_path / "world"))
    genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
    searches = oracle_searches(genome)
    kw = dict(searches=searches, aligner_factory=OracleAligner, log=lambda *_: None)
    base = str(tmp_path / "base")
    res = pipeline.run(paths["anchor"], paths["fq1"], paths["fq2"], paths["genome"], paths["gtf"], base, **kw)
    cands = res["BCRX"]
    assert cands
    anchor = [s.decode().upper() for _, s in pipeline.read_fasta(paths["anchor"])][0]
    index = ExonIndex.from_lines(open(paths["gtf"]).readlines())
    windows = filter_model.get_test_reads(cands, anchor, index, searches.getfasta)
    L = len(windows[0].split("\t")[0])
    torch.manual_seed(3)
    model = str(tmp_path / "model.pt")
    torch.save(filter_model.FusionFilter(L).double().state_dict(), model)
    missing = str(tmp_path / "missing")
    pipeline.run(paths["anchor"], paths["fq1"], paths["fq2"], paths["genome"], paths["gtf"], missing,
                 filt=dict(model_file=str(tmp_path / "nope.pt")), **kw)
    for t in TABLES:
        assert open(os.path.join(missing, "BCRX_fusion", t)).read() == open(os.path.join(base, "BCRX_fusion", t)).read()
    if len({len(w.split("\t")[0]) for w in windows}) > 1 or len(windows) < len(cands):
        raise AssertionError("the test world should give one window per candidate")
    torch.manual_seed(0)
    scored = str(tmp_path / "scored")
    pipeline.run(paths["anchor"], paths["fq1"], paths["fq2"], paths["genome"], paths["gtf"], scored,
                 filt=dict(model_file=model, device="cpu"), **kw)
    ab = [ln.rstrip("\n").split("\t") for ln in open(os.path.join(scored, "BCRX_fusion", TABLES[1]))]
    assert ab[0][5] == "Natural_score"
    for row in ab[1:]:
        assert 0.0 <= float(row[5]) <= 1.0
    assert os.path.exists(os.path.join(scored, "BCRX_fusion", "BCRX_fusion_test_reads.txt"))
