"""The multi-GPU product path (cli --gpus N) rehearsed on CPU: pipeline.run and singlecell.run
inside a gloo process group of 2 ranks, with the oracle backends.  The tables rank 0 writes
must equal the single-process run's byte for byte (S2 sharded on the chunk grid + the
candidate all-gatherv for bulk; cells dealt out to the ranks for single-cell).

Bulk input in BGZF is parsed in parts, one per rank (shard.read_pairs_sharded); plain gzip is
read whole by every rank.  The read-name columns list Python sets, as the reference does (functions.py Final_fusion), so
their order follows the interpreter's string hash seed: both runs are spawned with the same
PYTHONHASHSEED."""
import os
import socket

import torch.multiprocessing as mp

import afpkg  # noqa: F401
from anchored_fusion_amd import pipeline
from fusion_world import make_world

CHUNK = 300_000  # bases per bwa chunk in these runs: the sample spans several, both ranks align


def _backends(paths):
    from oracle_backends import OracleAligner, oracle_searches
    genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
    searches = oracle_searches(genome, CHUNK)
    return searches, (lambda a: OracleAligner(a, chunk_bases=CHUNK)), _discovery_factory(genome)


def _discovery_factory(genome):
    """The oracle as the per-rank dist_discover backend of a sharded run."""
    import oracle
    from oracle_discovery import OracleDiscovery, tiles_for
    og, tiles = oracle.OracleGenome(genome), tiles_for(genome)

    def make(anchor, reads, lens, lo, searches, gene):
        return OracleDiscovery(anchor.encode(), og, tiles, reads, lens, lo, CHUNK, gene)
    return make


def _worker(rank, world, port, paths, out, mode):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import torch.distributed as dist
    from anchored_fusion_amd import shard, singlecell
    shard.CHUNK_BASES = CHUNK
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    searches, factory, disc = _backends(paths)
    if mode == "bulk":
        pipeline.run(paths["anchor"], paths["fq1"], paths["fq2"], paths["genome"], paths["gtf"], out,
                     searches=searches, aligner_factory=factory, log=lambda *_: None, chunk_bases=CHUNK,
                     backend_factory=disc)
    else:
        singlecell.run(paths["anchor"], paths["cells"], paths["genome"], paths["gtf"], out, searches=searches,
                       aligner_factory=factory, batch_pairs=3000, log=lambda *_: None)
    dist.barrier()
    dist.destroy_process_group()


def _spawn(paths, out, mode, world=2):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    old = os.environ.get("PYTHONHASHSEED")
    os.environ["PYTHONHASHSEED"] = "7"
    try:
        mp.start_processes(_worker, args=(world, port, paths, out, mode), nprocs=world, join=True,
                           start_method="spawn")
    finally:
        if old is None:
            del os.environ["PYTHONHASHSEED"]
        else:
            os.environ["PYTHONHASHSEED"] = old


def test_pipeline_two_ranks_equals_single(tmp_path):
    paths, _ = make_world(str(tmp_path / "world"))
    one, two = str(tmp_path / "one"), str(tmp_path / "two")
    _spawn(paths, one, "bulk", world=1)
    _spawn(paths, two, "bulk")
    for t in ("BCRX_fusion_predictions.txt", "BCRX_fusion_predictions_abridged.txt"):
        a = open(os.path.join(one, "BCRX_fusion", t), "rb").read()
        b = open(os.path.join(two, "BCRX_fusion", t), "rb").read()
        assert a == b and len(a.splitlines()) > 1, t


def _bgzf_copy(paths, d):
    """The world's FASTQ pair rewritten as BGZF (bgzip's layout): the sharded ingest then splits it."""
    import gzip
    from multiprocessing import Pool

    from cells_world import write_bgzf
    os.makedirs(d, exist_ok=True)
    out = dict(paths)
    with Pool(4) as pool:
        for k in ("fq1", "fq2"):
            data = gzip.open(paths[k], "rb").read()
            out[k] = os.path.join(d, os.path.basename(paths[k]))
            write_bgzf(out[k], data, pool)
    return out


def test_pipeline_three_ranks_bgzf_equals_single(tmp_path):
    """BGZF input: each rank parses only its part of both files (sharded ingest), S2 on its whole
    chunks, the candidates' records / reads / names exchanged; rank 0's tables equal one process's."""
    paths, _ = make_world(str(tmp_path / "world"))
    paths = _bgzf_copy(paths, str(tmp_path / "bgzf"))
    one, three = str(tmp_path / "one"), str(tmp_path / "three")
    _spawn(paths, one, "bulk", world=1)
    _spawn(paths, three, "bulk", world=3)
    for t in ("BCRX_fusion_predictions.txt", "BCRX_fusion_predictions_abridged.txt"):
        a = open(os.path.join(one, "BCRX_fusion", t), "rb").read()
        b = open(os.path.join(three, "BCRX_fusion", t), "rb").read()
        assert a == b and len(a.splitlines()) > 1, t


def test_singlecell_two_ranks_equals_single(tmp_path):
    import shutil
    paths, _ = make_world(str(tmp_path / "world"))
    # three "cells": the sample's pairs split in thirds, gzip'd FASTQs named as SC:86-113 expects
    cells = tmp_path / "cells"
    from test_singlecell import _split_cells
    _split_cells(paths, str(cells), 3)
    paths = dict(paths, cells=str(cells))
    one, two = str(tmp_path / "one"), str(tmp_path / "two")
    _spawn(paths, one, "sc", world=1)
    _spawn(paths, two, "sc")
    for t in ("BCRX_fusion_gene_cell_predictions.txt", "BCRX_fusion_gene_cell_predictions_abridged.txt"):
        a = open(os.path.join(one, "BCRX", t), "rb").read()
        b = open(os.path.join(two, "BCRX", t), "rb").read()
        assert a == b, t
    shutil.rmtree(str(cells))


def test_cli_gpus_relaunches_under_torchrun(monkeypatch):
    """--gpus N (outside a launched job) starts N ranks under torch.distributed.run as a child
    process with the same flags, and returns its exit code."""
    import subprocess
    from anchored_fusion_amd import cli
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 3
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", fake_call)
    argv = ["--file_anchored_cds", "a.fa", "--file_ref_seq", "g.fa", "--file_ref_ann", "g.gtf", "--gpus", "4"]
    assert cli.main(argv) == 3
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-len(argv):] == argv
    assert cmd[-len(argv) - 1].endswith("run_anchored_fusion.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert cli.main_singlecell(["--file_anchored_cds", "a.fa", "--fastq_dir", "d", "--file_ref_seq", "g.fa",
                                "--file_ref_ann", "g.gtf", "--gpus", "2"]) == 3
    assert any(c.endswith("run_anchored_fusion_singlecell.py") for c in seen["cmd"])
