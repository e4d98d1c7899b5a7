"""The GPU side of the sharded S2 (shard.align_sharded) in a one-rank RCCL group: S2 on the
device, candidate rows packed on the device, the all-gatherv over RCCL, SparseCandidates.  The
gathered records must be the host API's records of the same pairs (a box has one GPU; the
two-rank split itself is covered by the gloo tests in test_shard.py / test_dist_pipeline.py)."""
import os
import socket

import numpy as np
import pytest

import afpkg  # noqa: F401


@pytest.mark.gpu
def test_align_sharded_rccl_one_rank(anchor):
    import torch
    import torch.distributed as dist
    from cases import synthetic_pairs
    from anchored_fusion_amd.align import AnchorAligner, partition
    from anchored_fusion_amd.shard import align_sharded
    reads, _, _ = synthetic_pairs(anchor, 20000, 150, seed=21)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        with AnchorAligner(anchor, device=0) as al:
            want = al.align_pairs(reads)
            sp = align_sharded(al, reads, None, 0, 1, device="cuda:0")
    finally:
        dist.destroy_process_group()
    got = sp.dense()
    for k in ("flag", "pos", "score", "n_cigar"):
        assert np.array_equal(getattr(got, k), getattr(want, k)), k
    live = np.arange(32)[None, :] < want.n_cigar[:, None]
    assert np.array_equal(np.where(live, got.cigar, 0), np.where(live, want.cigar, 0))
    for a, b in zip(sp.partition(), partition(want)):
        assert np.array_equal(a, b)
    assert 0 < len(sp.reads) < len(want.flag)
