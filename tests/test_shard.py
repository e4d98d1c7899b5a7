"""Multi-process (gloo, world size 2) test of the sharded S2 path on CPU: rank 0 reassembles
exactly the single-process records (oracle backend; the GPU backend has the same interface)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

import afpkg  # noqa: F401
from anchored_fusion_amd.shard import shard_range


def test_shard_ranges_cover():
    for n in (0, 1, 7, 49_999, 50_000, 50_001, 1_000_000):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert all(lo <= hi for lo, hi in spans)


def _worker(rank, world, port, path_in, path_out):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import torch.distributed as dist
    from oracle_backends import OracleAligner
    from anchored_fusion_amd.shard import align_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = np.load(path_in)
    res = align_sharded(OracleAligner(d["anchor"].tobytes()), d["reads"], None, rank, world, read_len=1_000_003)  # 4-pair chunks: both ranks work
    if rank == 0:
        np.savez(path_out, flag=res.flag, pos=res.pos, cigar=res.cigar, n_cigar=res.n_cigar)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_align_gloo(tmp_path, anchor):
    from cases import synthetic_pairs
    import oracle
    reads, _, _ = synthetic_pairs(anchor, 600000 // 100, 100, seed=5)  # 6,000 pairs
    path_in, path_out = str(tmp_path / "in.npz"), str(tmp_path / "out.npz")
    np.savez(path_in, anchor=np.frombuffer(anchor, dtype=np.uint8), reads=reads)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(2, port, path_in, path_out), nprocs=2, join=True, start_method="spawn")
    got = np.load(path_out)
    want = oracle.OracleIndex(anchor).align_pairs(reads, threads=4)
    for k in ("flag", "pos", "n_cigar", "cigar"):
        assert np.array_equal(got[k], want[k]), k
