"""Multi-process (gloo, world size 2) tests of the sharded S2 path on CPU: the same code the GPU
ranks run (device packing, counts + padded all_gather, SparseCandidates) on CPU tensors, with
the oracle aligner standing in for the GPU one.  Every rank must end with exactly the
single-process records and the same S3 partitions."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

import afpkg  # noqa: F401
from anchored_fusion_amd.shard import shard_pairs, shard_range


def test_shard_ranges_cover():
    for n in (0, 1, 7, 49_999, 50_000, 50_001, 1_000_000):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert all(lo <= hi for lo, hi in spans)


def test_shard_pairs_on_chunk_grid():
    """Uniform reads: shard_pairs == shard_range; ragged reads: every boundary is a bwa chunk end."""
    from anchored_fusion_amd.align import chunk_ends
    for n, L in ((1_000_000, 150), (70_001, 100), (5, 150)):
        for w in (1, 2, 8):
            assert [shard_pairs(np.full(n, 2 * L), r, w) for r in range(w)] == \
                [shard_range(n, r, w, L) for r in range(w)]
    rng = np.random.default_rng(3)
    pb = rng.integers(60, 300, size=200_000)
    ends = set(chunk_ends(pb, 10_000_000).tolist()) | {0}
    spans = [shard_pairs(pb, r, 3) for r in range(3)]
    assert spans[0][0] == 0 and spans[-1][1] == len(pb)
    assert all(lo in ends and hi in ends for lo, hi in spans)


def _worker(rank, world, port, path_in, path_out):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import torch.distributed as dist
    from oracle_backends import OracleAligner
    from anchored_fusion_amd.shard import align_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = np.load(path_in)
    lens = d["lens"] if d["lens"].size else None
    # 4 Mbase chunks: both ranks get whole chunks
    sp = align_sharded(OracleAligner(d["anchor"].tobytes()), d["reads"], lens, rank, world, chunk_bases=400_000)
    res = sp.dense()
    t1, t2, an = sp.partition()
    np.savez(path_out + f".{rank}.npz", flag=res.flag, pos=res.pos, score=res.score, cigar=res.cigar,
             n_cigar=res.n_cigar, hits=res.hits, t1=t1, t2=t2, an=an, nc=len(sp.reads))
    dist.barrier()
    dist.destroy_process_group()


def _run_world(tmp_path, anchor, reads, lens):
    path_in, path_out = str(tmp_path / "in.npz"), str(tmp_path / "out.npz")
    np.savez(path_in, anchor=np.frombuffer(anchor, dtype=np.uint8), reads=reads,
             lens=np.zeros(0, np.int32) if lens is None else lens)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(2, port, path_in, path_out), nprocs=2, join=True, start_method="spawn")
    return [np.load(path_out + f".{rank}.npz") for rank in range(2)]


def _check(got_all, want):
    from anchored_fusion_amd.align import AlignResult, partition
    res = AlignResult(**{k: want[k] for k in ("flag", "pos", "score", "n_cigar", "cigar", "hits")})
    parts = partition(res)
    for rank, got in enumerate(got_all):
        for k in ("flag", "pos", "score", "n_cigar"):
            assert np.array_equal(got[k], want[k]), (rank, k)
        # hits travel for candidate pairs; every other pair has none on either mate
        cand = (want["hits"].reshape(-1, 2) > 0).any(axis=1).repeat(2)
        assert np.array_equal(got["hits"][cand], want["hits"][cand]) and (got["hits"][~cand] == 0).all()
        assert (want["hits"][~cand] == 0).all()
        live = np.arange(32)[None, :] < want["n_cigar"][:, None]
        assert np.array_equal(np.where(live, got["cigar"], 0), np.where(live, want["cigar"], 0)), rank
        for k, p in zip(("t1", "t2", "an"), parts):
            assert np.array_equal(got[k], p), (rank, k)
        assert 0 < int(got["nc"]) < len(want["flag"])


def test_sharded_align_gloo(tmp_path, anchor):
    from cases import synthetic_pairs
    import oracle
    reads, _, _ = synthetic_pairs(anchor, 6000, 100, seed=5)  # 6,000 pairs, 1.2 Mbase: 3 chunks
    want = oracle.OracleIndex(anchor).align_pairs(reads, threads=4, chunk_bases=400_000)
    _check(_run_world(tmp_path, anchor, reads, None), want)


def test_sharded_align_gloo_ragged(tmp_path, anchor):
    """Ragged reads: shard boundaries follow the chunk ends of the actual lengths."""
    from cases import synthetic_pairs
    import oracle
    reads, _, _ = synthetic_pairs(anchor, 5000, 120, seed=9)
    rng = np.random.default_rng(9)
    lens = rng.integers(70, 121, size=reads.shape[0]).astype(np.int32)
    for r, ln in enumerate(lens):
        reads[r, ln:] = ord("N")
    want = oracle.OracleIndex(anchor).align_pairs(reads, lens, threads=4, chunk_bases=400_000)
    _check(_run_world(tmp_path, anchor, reads, lens), want)


def test_sparse_candidates_roundtrip(anchor):
    """Device packing (CPU tensors) -> SparseCandidates restores every record of the candidate
    pairs at any pair offset, and its partitions are the dense partitions."""
    import torch
    from cases import synthetic_pairs
    import oracle
    from anchored_fusion_amd.align import AlignResult, partition
    from anchored_fusion_amd.shard import SparseCandidates, pack_candidates_device
    reads, _, _ = synthetic_pairs(anchor, 3000, 100, seed=11)
    want = oracle.OracleIndex(anchor).align_pairs(reads, threads=4)
    out_t = {k: torch.from_numpy(np.ascontiguousarray(want[k], dtype=np.int32))
             for k in ("flag", "pos", "score", "n_cigar", "hits")}
    out_t["cigar"] = torch.from_numpy(np.ascontiguousarray(want["cigar"]).view(np.int32))
    for lo, total in ((0, 3000), (5000, 8000), ((1 << 31) + 7, (1 << 31) + 3007)):
        rows = pack_candidates_device(out_t, lo).numpy()
        assert 0 < len(rows) < 3000
        sp = SparseCandidates(rows, total)
        r = 2 * lo + np.arange(6000)
        for k in ("flag", "pos", "score", "n_cigar"):
            got = np.array([getattr(sp, k + "_at")(int(x)) for x in r[:200]]) if k in ("flag", "pos") else None
            if got is not None:
                assert np.array_equal(got, want[k][:200]), k
        dense_parts = partition(AlignResult(**{k: want[k] for k in ("flag", "pos", "score", "n_cigar", "cigar",
                                                                      "hits")}))
        for a, b in zip(sp.partition(), dense_parts):
            assert np.array_equal(a, b + 2 * lo)
        if total < 10_000:
            d = sp.dense()
            assert np.array_equal(d.flag[2 * lo:], want["flag"]) and (d.pos[:2 * lo] == -1).all()
