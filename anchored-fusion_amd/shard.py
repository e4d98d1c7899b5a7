"""Data-parallel S2 across GPUs (SURVEY.md §8 e).

One process per GPU. Rank r aligns the pairs in `shard_range(n, r, world)`, which are
contiguous and rounded to bwa's 10 Mbase chunk grid (SURVEY §8 e), with no data-path
collective. The one exchange step is an all-gatherv of the *breakpoint-candidate* records:
only pairs where a mate passed the seed filter (`hits > 0`, the K2 candidates, a few % of the
pairs) travel. Every other pair is, by construction of K3 (`csrc/align.hip` k_pairs), the
both-unmapped record (flag 0x1|0x4|0x8|mate bit, pos -1, score 0, no CIGAR, hits 0) and is
rebuilt locally. RCCL has no v-variant, so the gather is a counts all-gather followed by a
max-padded `all_gather` of int32 rows (torch.distributed: RCCL over xGMI for the "nccl"
backend, gloo in the CPU tests). Every rank ends with the full sample's records; rank 0 runs
S3-S8 on them.

Row payload per candidate pair: pair index (2 int32) + per mate flag, pos, score, n_cigar,
hits and 32 CIGAR words = 76 int32 (304 B).
"""
import numpy as np

from .align import AlignResult

CHUNK_BASES = 10_000_000   # bwa mem's batch size (-K default) the shard boundaries respect
ROW_WORDS = 2 + 2 * (5 + 32)


def chunk_pairs(read_len, chunk_bases=CHUNK_BASES):
    """Pairs per bwa input chunk when every read is read_len long."""
    return max(1, -(-chunk_bases // (2 * max(1, read_len))))


def shard_range(n_pairs, rank, world, read_len=100):
    """[lo, hi) of pairs for `rank`: contiguous, boundaries on the 10 Mbase chunk grid (bwa's
    bseq_read ends a chunk with the pair that brings it to >= CHUNK_BASES bases, so a chunk of
    uniform 2 x read_len pairs holds ceil(CHUNK_BASES / (2 read_len)) of them)."""
    chunk = chunk_pairs(read_len)
    n_chunks = (n_pairs + chunk - 1) // chunk
    per = [n_chunks // world + (1 if r < n_chunks % world else 0) for r in range(world)]
    lo = sum(per[:rank]) * chunk
    hi = min(n_pairs, lo + per[rank] * chunk)
    return min(lo, n_pairs), hi


def pack_candidates(res, lo):
    """Rows (int32 [k, ROW_WORDS]) of the pairs of `res` (pairs lo.. of the sample) where a mate
    has hits > 0."""
    hits = np.asarray(res.hits).reshape(-1, 2)
    sel = np.nonzero((hits > 0).any(axis=1))[0]
    k = len(sel)
    rows = np.zeros((k, ROW_WORDS), dtype=np.int32)
    gidx = sel.astype(np.int64) + lo
    rows[:, 0] = (gidx & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    rows[:, 1] = (gidx >> 32).astype(np.int32)
    c = 2
    for m in range(2):
        r = 2 * sel + m
        for f in (res.flag, res.pos, res.score, res.n_cigar, res.hits):
            rows[:, c] = np.asarray(f)[r]
            c += 1
        rows[:, c:c + 32] = np.asarray(res.cigar)[r]
        c += 32
    return rows


def unpack_candidates(rows, n_pairs):
    """Full AlignResult for n_pairs pairs: the rows' pairs as sent, every other pair the
    both-unmapped record K3 writes for reads without seed-filter hits."""
    n = 2 * n_pairs
    flag = np.empty(n, dtype=np.int32)
    flag[0::2] = 0x1 | 0x4 | 0x8 | 0x40
    flag[1::2] = 0x1 | 0x4 | 0x8 | 0x80
    pos = np.full(n, -1, dtype=np.int32)
    score = np.zeros(n, dtype=np.int32)
    n_cigar = np.zeros(n, dtype=np.int32)
    hits = np.zeros(n, dtype=np.int32)
    cigar = np.zeros((n, 32), dtype=np.uint32)
    if len(rows):
        gidx = rows[:, 0].view(np.uint32).astype(np.int64) | (rows[:, 1].astype(np.int64) << 32)
        c = 2
        for m in range(2):
            r = 2 * gidx + m
            for f in (flag, pos, score, n_cigar, hits):
                f[r] = rows[:, c]
                c += 1
            cigar[r] = rows[:, c:c + 32].view(np.uint32)
            c += 32
    return AlignResult(flag, pos, score, n_cigar, cigar, hits)


def allgatherv_rows(rows, group=None, device=None):
    """All-gather of a variable number of int32 rows per rank: counts first, then one
    max-padded all_gather (RCCL has no all-gatherv).  Returns the concatenation in rank order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = torch.device("cpu") if device is None else torch.device(device)
    t = torch.from_numpy(np.ascontiguousarray(rows)).to(dev)
    cnt = torch.tensor([t.shape[0]], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    counts = [int(c.item()) for c in cnts]
    mx = max(counts)
    if mx == 0:
        return np.zeros((0, rows.shape[1]), dtype=rows.dtype)
    pad = torch.zeros((mx, t.shape[1]), dtype=t.dtype, device=dev)
    pad[: t.shape[0]] = t
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return np.concatenate([b[:c].cpu().numpy() for b, c in zip(bufs, counts)])


def align_sharded(aligner, reads, lens, rank, world, group=None, read_len=100, device=None):
    """Every rank aligns its shard, then the candidate records are all-gathered: every rank
    returns the full AlignResult (its `hits` are carried for candidate pairs only; the rest
    are 0 by definition).  `device`: where the collective runs ("cuda:k" under RCCL)."""
    n_pairs = reads.shape[0] // 2
    lo, hi = shard_range(n_pairs, rank, world, read_len)
    if hi > lo:
        sub_lens = None if lens is None else lens[2 * lo:2 * hi]
        rows = pack_candidates(aligner.align_pairs(reads[2 * lo:2 * hi], sub_lens), lo)
    else:
        rows = np.zeros((0, ROW_WORDS), dtype=np.int32)
    return unpack_candidates(allgatherv_rows(rows, group, device), n_pairs)
