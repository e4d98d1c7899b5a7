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
    # all-gatherv: every rank holds the whole sample's records
    np.savez(path_out + f".{rank}.npz", flag=res.flag, pos=res.pos, score=res.score, cigar=res.cigar,
             n_cigar=res.n_cigar, hits=res.hits)
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
    want = oracle.OracleIndex(anchor).align_pairs(reads, threads=4)
    for rank in range(2):
        got = np.load(path_out + f".{rank}.npz")
        for k in ("flag", "pos", "score", "n_cigar", "hits"):
            assert np.array_equal(got[k], want[k]), (rank, k)
        live = np.arange(32)[None, :] < want["n_cigar"][:, None]
        assert np.array_equal(np.where(live, got["cigar"], 0), np.where(live, want["cigar"], 0)), rank


def test_candidate_rows_roundtrip(anchor):
    """pack -> unpack restores every record field of a shard (non-candidate pairs are the
    both-unmapped default), at any pair offset."""
    from cases import synthetic_pairs
    import oracle
    from anchored_fusion_amd.align import AlignResult
    from anchored_fusion_amd.shard import pack_candidates, unpack_candidates
    reads, _, _ = synthetic_pairs(anchor, 3000, 100, seed=11)
    want = oracle.OracleIndex(anchor).align_pairs(reads, threads=4)
    res = AlignResult(**{k: want[k] for k in ("flag", "pos", "score", "n_cigar", "cigar", "hits")})
    rows = pack_candidates(res, 0)
    assert 0 < len(rows) < 3000
    got = unpack_candidates(rows, 3000)
    for k in ("flag", "pos", "score", "n_cigar", "hits"):
        assert np.array_equal(getattr(got, k), want[k]), k
    # the same rows placed at a pair offset land at that offset
    big = unpack_candidates(pack_candidates(res, 5000), 8000)
    assert np.array_equal(big.flag[10000:], want["flag"]) and (big.hits[:10000] == 0).all()
