"""Sharded ingest (cli --gpus N): each rank parses its share of a BGZF FASTQ pair
(io.read_part, csrc/ingest.cpp af_fastq_part_*) and shard.read_pairs_sharded leaves every rank
whole bwa chunks of the sample (AF:182's input chunks).  Checked on CPU with gloo: the ranks'
pairs, in rank order, are exactly io.read_pairs' (names, bases, lengths), each rank's range
starts on the chunk grid of the whole input, and the ragged / multi-block / '@'-quality cases
parse as the whole-file reader does."""
import os
import socket
from multiprocessing import Pool

import numpy as np
import pytest
import torch.multiprocessing as mp

import afpkg  # noqa: F401
from anchored_fusion_amd import io as afio
from anchored_fusion_amd.align import chunk_ends
from cells_world import write_bgzf

CHUNK = 20_000  # bases per bwa chunk: the sample spans many chunks


def _write_pair(d, n, seed, bgzf=True, ragged=True, wrap=0):
    rng = np.random.default_rng(seed)
    recs = [[], []]
    for i in range(n):
        for m in range(2):
            L = int(rng.integers(60, 151)) if ragged else 100
            s = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, L)].tobytes().decode()
            q = "".join(chr(c) for c in rng.integers(33, 74, L))  # includes '@' (64) and '+' (43)
            if wrap:  # sequence and quality wrapped at `wrap` columns (kseq reads them; parts cannot split them)
                s = "\n".join(s[k:k + wrap] for k in range(0, len(s), wrap))
                q = "\n".join(q[k:k + wrap] for k in range(0, len(q), wrap))
            recs[m].append(f"@pair{i:07d}/{m + 1} extra\n{s}\n+\n{q}\n")
    paths = []
    with Pool(4) as pool:
        for m in range(2):
            p = os.path.join(d, f"r{m + 1}.fastq.gz")
            data = "".join(recs[m]).encode()
            if bgzf:
                write_bgzf(p, data, pool)
            else:
                import gzip
                with gzip.open(p, "wb") as fh:
                    fh.write(data)
            paths.append(p)
    return paths


def _worker(rank, world, port, fq1, fq2, out):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import torch.distributed as dist
    from anchored_fusion_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    names, reads, lens, lo, n_all = shard.read_pairs_sharded(fq1, fq2, rank, world, chunk_bases=CHUNK)
    ln = np.full(reads.shape[0], reads.shape[1], np.int32) if lens is None else lens
    np.savez(os.path.join(out, f"rank{rank}.npz"), names=np.array(list(names), dtype=object), reads=reads, lens=ln,
             lo=lo, n_all=n_all)
    dist.barrier()
    dist.destroy_process_group()


def _run(fq1, fq2, out, world):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(world, port, fq1, fq2, out), nprocs=world, join=True, start_method="spawn")
    return [np.load(os.path.join(out, f"rank{r}.npz"), allow_pickle=True) for r in range(world)]


def test_read_part_covers_file(tmp_path):
    fq1, _ = _write_pair(str(tmp_path), 3000, seed=1)
    names, reads, lens = afio.read_pairs(fq1, fq1)
    want = [names[i] for i in range(len(names))]
    for parts in (1, 2, 5, 17):
        got = [afio.read_part(fq1, p, parts) for p in range(parts)]
        assert sum(len(g[2]) for g in got) == len(want)
        assert [x for g in got for x in g[0]] == want
        L = np.concatenate([g[2] for g in got])
        assert np.array_equal(L, lens[0::2])
        k = 0
        for g in got:
            for i in range(len(g[2])):
                assert g[1][i, :g[2][i]].tobytes() == reads[2 * k, :lens[2 * k]].tobytes()
                k += 1


def test_read_part_rejects_plain_gzip(tmp_path):
    fq1, _ = _write_pair(str(tmp_path), 10, seed=2, bgzf=False)
    with pytest.raises(afio.NotBGZF):
        afio.read_part(fq1, 0, 2)


def test_read_part_rejects_wrapped_records(tmp_path):
    """Multi-line records: every part refuses (NotBGZF -> the whole-file reader), none drops records."""
    fq1, _ = _write_pair(str(tmp_path), 3000, seed=4, wrap=60)
    for parts in (1, 3):
        for p in range(parts):
            with pytest.raises(afio.NotBGZF):
                afio.read_part(fq1, p, parts)


@pytest.mark.parametrize("world,bgzf,wrap", [(2, True, 0), (3, True, 0), (2, False, 0), (3, True, 60)])
def test_read_pairs_sharded_gloo(tmp_path, world, bgzf, wrap):
    d = str(tmp_path)
    fq1, fq2 = _write_pair(d, 4000, seed=3, bgzf=bgzf, wrap=wrap)
    names, reads, lens = afio.read_pairs(fq1, fq2)
    lens = np.full(reads.shape[0], reads.shape[1], np.int32) if lens is None else lens
    grid = set(chunk_ends(lens.astype(np.int64).reshape(-1, 2).sum(axis=1), CHUNK).tolist()) | {0}
    res = _run(fq1, fq2, d, world)
    lo = 0
    for r, z in enumerate(res):
        assert int(z["n_all"]) == len(names)
        assert int(z["lo"]) == lo and lo in grid, (r, int(z["lo"]))
        k = len(z["names"])
        assert list(z["names"]) == [names[i] for i in range(lo, lo + k)]
        assert np.array_equal(z["lens"], lens[2 * lo:2 * (lo + k)])
        for i in range(2 * k):
            assert z["reads"][i, :z["lens"][i]].tobytes() == reads[2 * lo + i, :lens[2 * lo + i]].tobytes()
        lo += k
    assert lo == len(names)
