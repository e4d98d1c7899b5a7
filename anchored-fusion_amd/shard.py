"""Data-parallel S2 across GPUs (SURVEY.md §8 e).

One process per GPU (`torch.distributed`, RCCL over xGMI for the "nccl" backend; gloo in the
CPU tests).  Rank r aligns the pairs of its shard: whole bwa input chunks (10 Mbase each,
`chunk_ends` on the actual read lengths), contiguous, so every chunk's insert-size estimate is
the one a single `bwa mem` run makes (AF:182).  There is no data-path collective during S2.

The one exchange step is an all-gatherv of the *breakpoint-candidate* records, on device
tensors: K3 gives every pair without a seed-filter hit on either mate the both-unmapped record
(flag 0x1|0x4|0x8|mate bit, pos -1, score 0, no CIGAR), so only pairs where a mate has
`hits > 0` (a few % of the pairs) travel.  `pack_candidates_device` selects and packs them on
the device (torch ops on the current stream), `allgatherv_device` sends a counts all-gather and
then one max-padded `all_gather` (RCCL has no v-variant).  The result is a `SparseCandidates`:
the records of the candidate pairs only, with their global read indices; the S3 partitions of
the whole sample are exactly those of the candidate subset (every other read has pos -1 and
no filter keeps it), so no dense per-read array of the full sample is ever built.

Row payload per candidate pair: global pair index (2 int32) + per mate flag, pos, score,
n_cigar, hits and 32 CIGAR words = 76 int32 (304 B).  At configs[3] (50 M pairs over 8 GPUs,
~5 % candidate pairs at 2 x 150) that is ~0.3 M rows = ~95 MB per rank, ~0.76 GB gathered.
"""
import numpy as np

from .align import AlignResult, chunk_ends
from .align import partition as _partition_dense

CHUNK_BASES = 10_000_000   # bwa mem's batch size (-K default) the shard boundaries respect
ROW_WORDS = 2 + 2 * (5 + 32)
_FIELDS = ("flag", "pos", "score", "n_cigar", "hits")


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


def shard_pairs(pair_bases, rank, world, chunk_bases=CHUNK_BASES):
    """shard_range on the chunk boundaries of this input (ragged reads: `chunk_ends` of the
    per-pair base counts)."""
    ends = chunk_ends(pair_bases, chunk_bases)
    n_chunks = len(ends)
    per = [n_chunks // world + (1 if r < n_chunks % world else 0) for r in range(world)]
    c0 = sum(per[:rank])
    lo = int(ends[c0 - 1]) if c0 else 0
    hi = int(ends[c0 + per[rank] - 1]) if per[rank] else lo
    return lo, hi


def pack_candidates_device(out_t, lo):
    """Rows (int32 [k, ROW_WORDS], on out_t's device) of the pairs where a mate has hits > 0;
    out_t holds a shard's records (dict of [2n] int32 tensors + cigar [2n, 32]) whose first
    pair is pair `lo` of the sample."""
    import torch
    hits = out_t["hits"].view(-1, 2)
    sel = torch.nonzero((hits > 0).any(dim=1)).squeeze(1)
    g = sel + int(lo)
    cols = [g.to(torch.int32).unsqueeze(1), (g >> 32).to(torch.int32).unsqueeze(1)]
    cig = out_t["cigar"]
    if cig.dtype != torch.int32:
        cig = cig.view(torch.int32)
    for m in range(2):
        r = 2 * sel + m
        cols += [out_t[k].index_select(0, r).to(torch.int32).unsqueeze(1) for k in _FIELDS]
        cols.append(cig.index_select(0, r))
    return torch.cat(cols, dim=1).contiguous()


def allgatherv_device(rows_t, group=None):
    """All-gather of a variable number of rows per rank, on rows_t's device: counts first, then
    one max-padded all_gather.  Returns the concatenation in rank order (same device)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = rows_t.device
    cnt = torch.tensor([rows_t.shape[0]], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    counts = [int(c.item()) for c in cnts]
    mx = max(counts)
    if mx == 0:
        return rows_t.new_zeros((0, rows_t.shape[1]))
    pad = rows_t.new_zeros((mx, rows_t.shape[1]))
    pad[: rows_t.shape[0]] = rows_t
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)])


class SparseCandidates:
    """The S2 records of a whole sample held for its candidate pairs only (`reads` = global
    read indices, ascending, both mates of every candidate pair); every other read is the
    both-unmapped default.  The record API consume_gene uses (flag_at, pos_at, cigar_str,
    partition, n_mapped) matches AlignResult's."""

    def __init__(self, rows, n_pairs):
        rows = np.asarray(rows, dtype=np.int32).reshape(-1, ROW_WORDS)
        g = rows[:, 0].view(np.uint32).astype(np.int64) | (rows[:, 1].astype(np.int64) << 32)
        order = np.argsort(g, kind="stable")
        rows, g = rows[order], g[order]
        self.n_pairs, self.n_reads = int(n_pairs), 2 * int(n_pairs)
        k = len(g)
        self.reads = np.empty(2 * k, dtype=np.int64)
        self.reads[0::2], self.reads[1::2] = 2 * g, 2 * g + 1
        per = {f: np.empty(2 * k, dtype=np.int32) for f in _FIELDS}
        self.cigar = np.empty((2 * k, 32), dtype=np.uint32)
        c = 2
        for m in range(2):
            for f in _FIELDS:
                per[f][m::2] = rows[:, c]
                c += 1
            self.cigar[m::2] = rows[:, c:c + 32].view(np.uint32)
            c += 32
        self.flag, self.pos, self.score, self.n_cigar, self.hits = (per[f] for f in _FIELDS)
        self._sub = AlignResult(self.flag, self.pos, self.score, self.n_cigar, self.cigar, self.hits)

    def __len__(self):
        return self.n_reads

    def _row(self, r):
        i = int(np.searchsorted(self.reads, r))
        return i if i < len(self.reads) and self.reads[i] == r else -1

    def flag_at(self, r):
        i = self._row(r)
        return int(self.flag[i]) if i >= 0 else (0x1 | 0x4 | 0x8 | (0x40 if r % 2 == 0 else 0x80))

    def pos_at(self, r):
        i = self._row(r)
        return int(self.pos[i]) if i >= 0 else -1

    def cigar_str(self, r):
        i = self._row(r)
        return "*" if i < 0 else self._sub.cigar_str(i)

    def n_mapped(self):
        return int(((self.flag & 4) == 0).sum())

    def partition(self):
        """align.partition of the whole sample: the candidate subset in samtools order (ties in
        input order = ascending global index, as `reads` is), mapped to global read indices."""
        return tuple(self.reads[p] for p in _partition_dense(self._sub))

    def dense(self):
        """The full-sample AlignResult (tests; O(n_reads) memory)."""
        n = self.n_reads
        flag = np.empty(n, dtype=np.int32)
        flag[0::2] = 0x1 | 0x4 | 0x8 | 0x40
        flag[1::2] = 0x1 | 0x4 | 0x8 | 0x80
        out = AlignResult(flag, np.full(n, -1, np.int32), np.zeros(n, np.int32), np.zeros(n, np.int32),
                          np.zeros((n, 32), np.uint32), np.zeros(n, np.int32))
        for f in _FIELDS:
            getattr(out, f)[self.reads] = getattr(self, f)
        out.cigar[self.reads] = self.cigar
        return out


def _shard_records_t(aligner, reads, lens, lo, hi, device):
    """S2 of pairs [lo, hi) -> dict of record tensors: on the GPU (align_pairs_device, the
    reads copied once from pinned host memory) when the aligner has a device path and device is
    a GPU; otherwise the host result as CPU tensors (the gloo tests' oracle aligner)."""
    import torch
    sub = reads[2 * lo:2 * hi]
    sub_lens = None if lens is None else np.ascontiguousarray(lens[2 * lo:2 * hi], dtype=np.int32)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda" and hasattr(aligner, "align_pairs_device"):
        n = hi - lo
        reads_t = torch.from_numpy(np.ascontiguousarray(sub)).pin_memory().to(dev, non_blocking=True)
        lens_t = None if sub_lens is None else torch.from_numpy(sub_lens).to(dev)
        out_t = {k: torch.zeros(2 * n, dtype=torch.int32, device=dev) for k in _FIELDS}
        out_t["cigar"] = torch.zeros((2 * n, 32), dtype=torch.int32, device=dev)
        aligner.align_pairs_device(reads_t, n, reads_t.shape[1], out_t, lens_t=lens_t,
                                   stream=torch.cuda.current_stream(dev), pair_base=lo)
        return out_t
    res = aligner.align_pairs(sub, sub_lens, pair_base=lo) if _takes_pair_base(aligner) else \
        aligner.align_pairs(sub, sub_lens)
    out = {k: torch.from_numpy(np.ascontiguousarray(getattr(res, k), dtype=np.int32)) for k in _FIELDS}
    out["cigar"] = torch.from_numpy(np.ascontiguousarray(res.cigar).view(np.int32))
    return {k: v.to(dev) for k, v in out.items()}


def _takes_pair_base(aligner):
    import inspect
    try:
        return "pair_base" in inspect.signature(aligner.align_pairs).parameters
    except (TypeError, ValueError):
        return False


def align_sharded(aligner, reads, lens, rank, world, group=None, device=None, chunk_bases=None):
    """Every rank runs S2 on its shard, packs the candidate pairs on the device and joins the
    all-gatherv: every rank returns the whole sample's SparseCandidates.  device: the rank's GPU
    ("cuda:k", RCCL) or None / "cpu" (gloo)."""
    import torch
    n_pairs = reads.shape[0] // 2
    if lens is None:
        pair_bases = np.full(n_pairs, 2 * reads.shape[1], dtype=np.int64)
    else:
        pair_bases = np.asarray(lens, dtype=np.int64).reshape(-1, 2).sum(axis=1)
    lo, hi = shard_pairs(pair_bases, rank, world, CHUNK_BASES if chunk_bases is None else chunk_bases)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if hi > lo:
        rows_t = pack_candidates_device(_shard_records_t(aligner, reads, lens, lo, hi, dev), lo)
    else:
        rows_t = torch.zeros((0, ROW_WORDS), dtype=torch.int32, device=dev)
    return SparseCandidates(allgatherv_device(rows_t, group).cpu().numpy(), n_pairs)
