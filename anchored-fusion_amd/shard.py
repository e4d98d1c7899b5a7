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
from .io import Names, NotBGZF, read_pairs, read_part
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


def _shard_records_t(aligner, reads, lens, lo, hi, device, pair_base=None):
    """S2 of pairs [lo, hi) of `reads` (the sample's pairs from pair_base, default lo) -> dict of
    record tensors: on the GPU (align_pairs_device, the reads copied once from pinned host
    memory) when the aligner has a device path and device is a GPU; otherwise the host result as
    CPU tensors (the gloo tests' oracle aligner)."""
    import torch
    pb = lo if pair_base is None else int(pair_base)
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
                                   stream=torch.cuda.current_stream(dev), pair_base=pb)
        return out_t
    res = aligner.align_pairs(sub, sub_lens, pair_base=pb) if _takes_pair_base(aligner) else \
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


# ---- sharded ingest (each rank parses its share of a BGZF FASTQ pair) -----------------------------

def _pack(names, seqs, lens):
    """Rows (names Names [k], seqs uint8 [r, w], lens int32 [r]) as one uint8 payload."""
    k, r = len(names), seqs.shape[0]
    w = seqs.shape[1] if r else 1
    nm = [names[i].encode() + b"\0" for i in range(k)]
    arena = b"".join(nm)
    off = np.zeros(k, np.int64)
    if k > 1:
        off[1:] = np.cumsum([len(x) for x in nm])[:-1]
    head = np.array([k, r, w, len(arena)], np.int64)
    return np.concatenate([head.view(np.uint8), off.view(np.uint8), np.frombuffer(arena, np.uint8),
                           np.ascontiguousarray(lens, np.int32).view(np.uint8),
                           np.ascontiguousarray(seqs, np.uint8).reshape(-1)])


def _unpack(buf):
    k, r, w, na = (int(v) for v in buf[:32].view(np.int64))
    o = 32
    off = buf[o:o + 8 * k].view(np.int64).copy()
    o += 8 * k
    arena = buf[o:o + na].tobytes()
    o += na
    lens = buf[o:o + 4 * r].view(np.int32).copy()
    o += 4 * r
    seqs = buf[o:o + r * w].reshape(r, w) if r else np.zeros((0, w), np.uint8)
    return Names(arena, off), seqs, lens


_EMPTY = (Names(b"", np.zeros(0, np.int64)), np.zeros((0, 1), np.uint8), np.zeros(0, np.int32))


def _exchange(payloads, group):
    """payloads[d] (uint8 numpy) to rank d, for every d; returns the payload from every rank
    (point-to-point over `group`, a CPU (gloo) group: sizes first, then the bytes)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    got = [None] * world
    got[rank] = payloads[rank]
    for step in range(1, world):
        dst, src = (rank + step) % world, (rank - step) % world
        out_t = torch.from_numpy(np.ascontiguousarray(payloads[dst]))
        sz = torch.tensor([out_t.numel()], dtype=torch.int64)
        rsz = torch.zeros(1, dtype=torch.int64)
        for q in (dist.isend(sz, _global(dst, group), group=group), dist.irecv(rsz, _global(src, group), group=group)):
            q.wait()
        rbuf = torch.empty(int(rsz.item()), dtype=torch.uint8)
        reqs = [dist.isend(out_t, _global(dst, group), group=group)] if out_t.numel() else []
        if rbuf.numel():
            reqs.append(dist.irecv(rbuf, _global(src, group), group=group))
        for q in reqs:
            q.wait()
        got[src] = rbuf.numpy()
    return got


def _global(r, group):
    import torch.distributed as dist
    return r if group is None else dist.get_global_rank(group, r)


def _gather_ints(vals, group):
    import torch
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.int64)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return np.stack([o.numpy() for o in out])


def _cat_rows(parts):
    """Concatenation of (names, seqs, lens) parts (rows padded to the widest)."""
    parts = [p for p in parts if p[2].size]
    if not parts:
        return _EMPTY
    w = max(p[1].shape[1] for p in parts)
    rows = np.full((sum(p[1].shape[0] for p in parts), w), ord("N"), np.uint8)
    r = 0
    for p in parts:
        rows[r:r + p[1].shape[0], :p[1].shape[1]] = p[1]
        r += p[1].shape[0]
    return Names.concat([p[0] for p in parts]), rows, np.concatenate([p[2] for p in parts])


def chunk_carry(bases, s_in, owner, rank, chunk_bases):
    """bwa's chunking (bseq_read: a chunk ends with the pair that brings it to >= chunk_bases
    bases) continued over one rank's pairs.  (s_in, owner): the bases of the chunk still open at
    this rank's first pair and the rank it started on (owner -1: none).  Returns (head, s_out,
    owner_out): the leading pairs that belong to the open chunk and the chunk open after the
    last pair."""
    n = len(bases)
    cum = np.cumsum(np.asarray(bases, dtype=np.int64))
    head = 0
    if owner >= 0:
        e = int(np.searchsorted(cum, chunk_bases - s_in, side="left"))
        if e >= n:
            return n, s_in + (int(cum[-1]) if n else 0), owner
        head = e + 1
    rest = np.asarray(bases[head:], dtype=np.int64)
    if rest.size == 0:
        return head, 0, -1
    ends = chunk_ends(rest, chunk_bases)
    last0 = int(ends[-2]) if len(ends) > 1 else 0
    tail = int(rest[last0:].sum())
    return (head, 0, -1) if tail >= chunk_bases else (head, tail, rank)


def read_pairs_sharded(fq1, fq2, rank, world, group=None, chunk_bases=CHUNK_BASES, threads=0):
    """This rank's whole bwa chunks of a FASTQ pair, each rank parsing only its share of BGZF
    input: returns (names, reads [2n, stride], lens [2n] or None, lo, n_pairs_total) for the
    pairs [lo, lo + n) of the sample -- contiguous, on the chunk grid of the whole input, so every
    chunk's insert-size estimate and read ids are those of one `bwa mem` run (AF:182).

    Each rank reads part `rank` of both files (io.read_part: the records whose header starts in
    its share of the BGZF blocks).  The record counts are all-gathered; every mate 2 goes to the
    rank holding its mate 1 (point-to-point over `group`, a CPU group); bwa's chunking is carried
    from rank to rank (chunk_carry), and the pairs that close a chunk opened on an earlier rank
    move to that rank.  Input that is not BGZF is read whole by every rank and sliced
    (shard_pairs).  world == 1: read_pairs."""
    if world == 1:
        names, reads, lens = read_pairs(fq1, fq2, threads=threads)
        return names, reads, lens, 0, reads.shape[0] // 2
    import torch
    import torch.distributed as dist
    try:
        p1, p2 = read_part(fq1, rank, world, threads), read_part(fq2, rank, world, threads)
        ok = 1
    except NotBGZF:
        ok = 0
    if not _gather_ints([ok], group).all():
        names, reads, lens = read_pairs(fq1, fq2, threads=threads)
        n_all = reads.shape[0] // 2
        pb = np.full(n_all, 2 * reads.shape[1], np.int64) if lens is None else \
            np.asarray(lens, np.int64).reshape(-1, 2).sum(axis=1)
        lo, hi = shard_pairs(pb, rank, world, chunk_bases)
        return names.slice(lo, hi), reads[2 * lo:2 * hi], None if lens is None else lens[2 * lo:2 * hi], lo, n_all
    cnt = _gather_ints([len(p1[2]), len(p2[2])], group)
    o1 = np.concatenate([[0], np.cumsum(cnt[:, 0])]).astype(np.int64)
    o2 = np.concatenate([[0], np.cumsum(cnt[:, 1])]).astype(np.int64)
    if o1[-1] != o2[-1]:
        raise ValueError(f"paired FASTQs differ in length: {int(o1[-1])} vs {int(o2[-1])} records")
    n_all = int(o1[-1])
    # every mate 2 to the rank that holds its mate 1
    pay = []
    for d in range(world):
        a = int(max(o1[d], o2[rank]) - o2[rank])
        b = int(min(o1[d + 1], o2[rank + 1]) - o2[rank])
        a, b = max(a, 0), max(b, 0)
        pay.append(_pack(p2[0].slice(a, b) if b > a else _EMPTY[0], p2[1][a:b] if b > a else _EMPTY[1],
                         p2[2][a:b] if b > a else _EMPTY[2]))
    n2, s2, l2 = _cat_rows([_unpack(x) for x in _exchange(pay, group)])
    n1, s1, l1 = p1
    n = len(l1)
    if len(l2) != n:
        raise RuntimeError("sharded ingest: the mate exchange lost records")
    for i in range(n):
        if n1[i] != n2[i]:  # bwa: "paired reads have different names"
            raise ValueError(f'paired reads have different names: "{n1[i]}", "{n2[i]}"')
    w = max(s1.shape[1], s2.shape[1])
    reads = np.full((2 * n, w), ord("N"), np.uint8)
    reads[0::2, :s1.shape[1]] = s1
    reads[1::2, :s2.shape[1]] = s2
    lens = np.empty(2 * n, np.int32)
    lens[0::2], lens[1::2] = l1, l2
    # bwa's chunks, carried from rank to rank: (open chunk's bases, the rank it started on)
    carry = torch.tensor([0, -1], dtype=torch.int64)
    if rank > 0:
        dist.recv(carry, _global(rank - 1, group), group=group)
    s_in, owner = int(carry[0]), int(carry[1])
    head, s_out, own_out = chunk_carry(lens.reshape(-1, 2).astype(np.int64).sum(axis=1), s_in, owner, rank,
                                       chunk_bases)
    if rank + 1 < world:
        dist.send(torch.tensor([s_out, own_out], dtype=torch.int64), _global(rank + 1, group), group=group)
    # the leading pairs close a chunk opened on rank `owner`: they move there
    pay = [_pack(*_EMPTY)] * world
    if head:
        pay = list(pay)
        pay[owner] = _pack(n1.slice(0, head), reads[:2 * head], lens[:2 * head])
    got = _exchange(pay, group)
    mine = (n1.slice(head, n), reads[2 * head:], lens[2 * head:])
    names, reads, lens = _cat_rows([mine] + [_unpack(got[src]) for src in range(rank + 1, world)])
    lo = int(o1[rank]) + head
    if reads.shape[0]:
        reads = np.ascontiguousarray(reads[:, :max(1, int(lens.max()))])
    return names, reads, (None if (lens == reads.shape[1]).all() else lens), lo, n_all
