"""bench.py's host-side legs on CPU (the driver runs bench.py only on the GPU box): the configs[2]
CPU baseline (cpu_baseline_c3: the oracle over S2 + S3 + gathers + S4/S5 + S5 check + S6 on a
bounded sample) runs on a small fusion world and reports every stage, and genome_subset cuts the
gene loci +- flank out of a world's contigs."""
import types

import numpy as np
import torch

import afpkg  # noqa: F401
import bench
from anchored_fusion_amd import io as afio
from anchored_fusion_amd import pipeline
from fusion_world import make_world


def test_cpu_baseline_c3_runs_every_stage(tmp_path):
    paths, _ = make_world(str(tmp_path / "w"), n_fusion=400, n_anchor=300, n_background=800)
    names, reads, lens = afio.read_pairs(paths["fq1"], paths["fq2"])
    subset = [(h.split()[0], s.upper()) for h, s in pipeline.read_fasta(paths["genome"])]
    anchor = afio.anchor_sequence(paths["anchor"])
    args = types.SimpleNamespace(cpu_sample=1000, cpu_seconds=0.5, cpu_threads=2)
    out = bench.cpu_baseline_c3(anchor, torch.from_numpy(reads), args, subset)
    assert out["value"] > 0 and out["cores"] == 2 and out["kind"] == "port"
    assert set(out["stages_s_per_pass"]) == {"s2_s3", "gather", "s4", "s5", "s5_check", "s6"}
    q = out["queries_per_pass"]
    assert q["s4_pairs"] > 0 and q["s5_split_reads"] > 0 and q["s6_queries"] > 0, q


def test_genome_subset_windows():
    W = types.SimpleNamespace(names=["c1", "c2"], lens=[10_000, 5_000], offsets=[0, 10_512],
                              loci={"anchor": [("c1", 1000, 1200), ("c1", 3000, 3300)],
                                    "p0": [("c2", 4700, 4900)]})
    blob = np.frombuffer(b"A" * 10_000 + b"N" * 512 + b"C" * 5_000, np.uint8)
    W.blob = torch.from_numpy(blob.copy())
    sub = bench.genome_subset(W, flank=500)
    # the anchor's exons on c1 -> one window (500 .. 3800); the partner's on c2 clipped at its end
    assert [n for n, _ in sub] == ["c1:500-3800", "c2:4200-5000"]
    assert sub[0][1] == b"A" * 3300 and sub[1][1] == b"C" * 800
