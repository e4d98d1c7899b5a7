"""Data-parallel S2 across GPUs (SURVEY.md §8 e).

One process per GPU. Rank r aligns the pairs in `shard_range(n, r, world)`, which are
contiguous and rounded to bwa's 10 Mbase chunk grid (SURVEY §8 e), with no data-path
collective. The small per-read records then travel to rank 0 in one gather (torch.distributed:
RCCL on GPUs, gloo in the CPU tests), and rank 0 runs S3-S8 on the whole sample.

The payload is the per-read record fields: 4 int32 plus 32 CIGAR words. Under 0.2 KB per
read, it is a small fraction of the 2·L read bytes each rank streamed.
"""
import numpy as np

from .align import AlignResult

CHUNK_BASES = 10_000_000   # bwa mem's batch size (-K default) the shard boundaries respect


def shard_range(n_pairs, rank, world, read_len=100):
    """[lo, hi) of pairs for `rank`: contiguous, boundaries on the 10 Mbase chunk grid."""
    chunk = max(1, CHUNK_BASES // (2 * max(1, read_len)))
    n_chunks = (n_pairs + chunk - 1) // chunk
    per = [n_chunks // world + (1 if r < n_chunks % world else 0) for r in range(world)]
    lo = sum(per[:rank]) * chunk
    hi = min(n_pairs, lo + per[rank] * chunk)
    return min(lo, n_pairs), hi


def align_sharded(aligner, reads, lens, rank, world, group=None, read_len=100):
    """Every rank aligns its shard; rank 0 returns the full AlignResult (others None)."""
    import torch.distributed as dist
    n_pairs = reads.shape[0] // 2
    lo, hi = shard_range(n_pairs, rank, world, read_len)
    part = None
    if hi > lo:
        sub_lens = None if lens is None else lens[2 * lo:2 * hi]
        r = aligner.align_pairs(reads[2 * lo:2 * hi], sub_lens)
        part = (lo, r.flag, r.pos, r.score, r.n_cigar, r.cigar, r.hits)
    parts = [None] * world if rank == 0 else None
    dist.gather_object(part, parts, dst=0, group=group)
    if rank != 0:
        return None
    parts = sorted((p for p in parts if p is not None), key=lambda p: p[0])
    cat = [np.concatenate([p[k] for p in parts]) for k in range(1, 7)]
    return AlignResult(*cat)
