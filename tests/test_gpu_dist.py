"""The GPU backend of dist_discover (discover.CandidateDiscovery's local_phase / s5_s6_phase /
s4_phase, the form every rank of a multi-GPU run takes) on one GPU: its texts -- S4's SAM lines,
the split_sam lines S5's check keeps, S6's PSL -- equal the one-process host path over the CPU
oracle (pipeline.host_products with the oracle searches), byte for byte."""
import numpy as np
import pytest

import afpkg  # noqa: F401
from anchored_fusion_amd import pipeline
from fusion_world import make_world

pytestmark = pytest.mark.gpu

CHUNK = 300_000
GENE = "BCRX"


@pytest.mark.parametrize("collectives", [False, True])
def test_gpu_backend_equals_oracle_host_path(tmp_path, monkeypatch, collectives):
    """collectives: the step's exchanges (the S5 keys' all-gathers, S4's read all-to-alls, the
    record / survivor / S6-row gathers to rank 0 as all-to-alls with one destination) run through
    a one-rank RCCL group on device tensors (AF_DIST_COLLECTIVES=1) instead of the world-1
    shortcut -- the same texts."""
    import os
    import socket

    import torch
    import torch.distributed as dist
    from anchored_fusion_amd import dist_discover
    from anchored_fusion_amd import io as afio
    from oracle_backends import OracleAligner, oracle_searches
    paths, _ = make_world(str(tmp_path / "world"), n_fusion=600, n_anchor=500, n_background=2500)
    names, reads, lens = afio.read_pairs(paths["fq1"], paths["fq2"])
    genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
    anchor = afio.anchor_sequence(paths["anchor"]).decode()
    res = OracleAligner(anchor.encode(), chunk_bases=CHUNK).align_pairs(reads, lens)
    want = pipeline.host_products(GENE, names, reads, lens, res, oracle_searches(genome, CHUNK), log=lambda *_: None)
    searches = pipeline.Searches(genome, device=0, chunk_bases=CHUNK)
    backend = pipeline.gpu_backend(0, CHUNK)(anchor, reads, lens, 0, searches, GENE)
    if collectives:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        monkeypatch.setenv("AF_DIST_COLLECTIVES", "1")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        out, counts = dist_discover.search(backend, 0, 0, 1, device="cuda:0", names=names, s4_reads=True)
        got = dist_discover.render(out, backend, GENE, [n for n, _ in genome])
        torch.cuda.synchronize()
    finally:
        backend.close()
        if collectives:
            dist.destroy_process_group()
    assert counts["s6_queries"] > 10 and len(want[1]) > 10
    for g, w, what in zip(got, want, ("S4 SAM", "split_sam", "S6 PSL")):
        assert list(g) == list(w), what
