"""S3-S6 of a sample sharded over GPUs, each rank on its own reads, with the global order of one
`bwa mem` run (SURVEY.md §8 e).

After S2 on its whole bwa chunks (pairs lo .. lo + n of the sample), every rank holds the
anchored records of its reads.  The reference's later stages read files in coordinate order
over the WHOLE sample, and three things depend on that order:

* S4 (`bwa mem -M genome tmp1.fq tmp2.fq`, AF:188) pairs the k-th record of the sorted tmp1 list
  with the k-th of tmp2, and estimates insert sizes per input chunk of that stream;
* S5 (`bwa mem -M genome split.fa`, functions.py:716) breaks ties between equal-scoring
  alignments with hash_64 of each read's ordinal in split.fa;
* the genome check (fn:718-768) groups records by consecutive QNAME.

So the ranks all-gather the sort keys of their tmp1 / tmp2 / split-read lists (samtools' key:
2 pos + strand, ties by the global read row -- the rank order), which gives every rank each of
its split reads' global ordinal and whether its predecessor in the global order has the same
QNAME (then both are mates of one pair, on the same rank).  S5, its check and S6 then run on
every rank over its own queries with those ids and group flags (`af_genome_align_se_ids_device`,
`af_s5_filter_device` with d_cont).  S4's input stream -- tmp1 / tmp2 zipped in the global order
-- is known to every rank from the keys alone; each rank aligns whole bwa chunks of it
(`pair_base` = its first pair, so read ids and insert-size chunks are those of one run), the
reads of its share sent to it by their owners (one all-to-all), and the compacted records go to
rank 0.  The survivors and their S6 rows go to rank 0 too, ordered there by ordinal.  `search`
stops there (the bench step); `render` turns the result into what `pipeline.consume_products`
reads, equal to the one-process run's byte for byte (tests/test_dist_discover.py).

Everything is a torch tensor on `device` from the backend's phases to the collectives: on GPUs
the lists never leave HBM (RCCL all-gathers / all-to-alls over xGMI); the gloo tests run the
same code on CPU tensors.  The per-rank work is done by a backend with three phases --
`local_phase` (S2 + S3 + the gathers), `s5_s6_phase(ids, cont)` and `s4_phase(q, ql, pair_base)`
-- implemented by discover.CandidateDiscovery on the GPU; the tests run the CPU oracle through
the same driver.  Read names (for `render` only) go over `host_group` as objects.
"""
import os

import numpy as np

from .genome import sam_lines

PSL_HEADER = ["psLayout version 3\n", "\n"]
_OPS = "MIDNSHP=X"
PSL_WORDS = 82  # af_psl / blat.PSL_DTYPE as int32 words (328 B)


def cigar_string(words, n):
    return "".join(f"{int(v) >> 4}{_OPS[int(v) & 15]}" for v in words[:int(n)])


class LocalQueries:
    """A rank's lists after S2 + S3 + the gathers (tensors on the rank's device, or numpy arrays;
    rows are local read rows).

    t1 / t2: the tmp1 / tmp2 rows in samtools order with their keys (2 pos + strand) and the reads
    as sequenced (seq uint8 [k, w], len int32 [k]: bytes past a row's length are ignored); s5: the
    split reads (the S5 queries) in order with keys, the anchored record's POS and CIGAR (cigar
    int32 words [k, 32], ncig), and the queries' SEQ in SAM orientation (seq uint8 [k, w], len).

    A backend's s5_s6_phase(ids, cont) (int64 / uint8 tensors on the device) returns dict(src
    [m]: the survivors' S5 indices, s6_seq uint8 [m, w] + s6_len [m]: their S6 queries, psl int32
    words [m, MAX_ROWS, 82] (af_psl rows) + n_psl [m]); s4_phase(q uint8 [2 P, w], ql [2 P],
    pair_base) returns (af_grec rows as int32 words [2 P, MAX_REC, 44], counts [2 P])."""

    def __init__(self, t1, t2, s5):
        self.t1, self.t2, self.s5 = t1, t2, s5


# ---- tensor helpers ---------------------------------------------------------------------------
def _t(x, dev, dtype=None):
    import torch
    t = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t.to(dev).contiguous()


def _words(t):
    """Rows of t (any dtype, [n] or [n, ...]) as int32 words [n, w]."""
    import torch
    n = int(t.shape[0])
    per = t.element_size() * (int(np.prod(t.shape[1:])) if t.dim() > 1 else 1)
    if t.numel() == 0:
        return torch.zeros((n, per // 4), dtype=torch.int32, device=t.device)
    return t.contiguous().view(torch.uint8).reshape(n, per).view(torch.int32)


def _i64(w):
    """int32 word pairs [n, 2] -> int64 [n]."""
    import torch
    return w.contiguous().view(torch.int64).reshape(-1)


def _order(keys, rows):
    """The global order of concatenated per-rank lists: by key, ties by global row."""
    import torch
    o = torch.argsort(rows, stable=True)
    return o[torch.argsort(keys[o], stable=True)]


def _width(lens):
    """Row width for sequences of these lengths: the longest, at least 1, a multiple of 4."""
    w = max(1, int(lens.max()) if lens.numel() else 1)
    return -(-w // 4) * 4


def _block(seq, lens, idx, width):
    """Rows idx of seq (uint8 [k, w]) as uint8 [len(idx), width], 'N' past each row's length."""
    import torch
    dev = seq.device
    out = torch.full((int(idx.numel()), width), ord("N"), dtype=torch.uint8, device=dev)
    if idx.numel():
        w = min(width, int(seq.shape[1]))
        out[:, :w] = seq[idx, :w]
        out[torch.arange(width, device=dev)[None, :] >= lens[idx][:, None]] = ord("N")
    return out


def _collective(world):
    """Whether the exchanges go through the process group: always at world > 1; at world 1 only
    when AF_DIST_COLLECTIVES=1 and a group is initialised (a one-rank RCCL group runs the same
    all-gathers / all-to-alls on one GPU -- tests/test_gpu_dist.py), else the local shortcut."""
    if world > 1:
        return True
    import torch.distributed as dist
    return os.environ.get("AF_DIST_COLLECTIVES") == "1" and dist.is_available() and dist.is_initialized()


def _allgatherv(t, group, world):
    """All-gatherv of the rows of t (any dtype) over group; world 1: t itself."""
    import torch

    from .shard import allgatherv_device
    if not _collective(world):
        return t
    b = _words(t).view(torch.uint8)
    out = allgatherv_device(b, group)
    return out.view(t.dtype).reshape(-1, *t.shape[1:])


def _alltoallv(parts, recv_rows, group, world):
    """parts[d]: the rows (uint8 [n_d, per], same per everywhere) this rank sends to rank d;
    recv_rows[s]: how many rows rank s sends here.  Returns the received rows in rank order."""
    import torch
    import torch.distributed as dist
    per = int(parts[0].shape[1])
    inp = torch.cat(parts).contiguous()
    if not _collective(world):
        return inp
    out = torch.empty((int(sum(recv_rows)), per), dtype=torch.uint8, device=inp.device)
    dist.all_to_all_single(out.view(-1), inp.view(-1), [int(r) * per for r in recv_rows],
                           [int(p.shape[0]) * per for p in parts], group=group)
    return out


def _gatherv(t, group, world, rank):
    """The rows of t from every rank on rank 0 (rank order), None elsewhere (an all-to-all whose
    only destination is rank 0)."""
    import torch
    if not _collective(world):
        return t
    b = _words(t).view(torch.uint8)
    n = _allgatherv(torch.tensor([[b.shape[0]]], dtype=torch.int64, device=b.device), group, world)[:, 0].tolist()
    parts = [b if d == 0 else b[:0] for d in range(world)]
    out = _alltoallv(parts, n if rank == 0 else [0] * world, group, world)
    return out.view(t.dtype).reshape(-1, *t.shape[1:]) if rank == 0 else None


# ---- the distributed step ---------------------------------------------------------------------
def search(backend, lo, rank, world, group=None, device="cpu", names=None, host_group=None, s4_reads=False):
    """The distributed S3-S6 of one gene (backend already holds this rank's S2 input).  Returns,
    on rank 0, dict(s4=(pair reads or None, lens, records, counts, t1 global rows), surv=(the
    survivors' rows by ordinal), psl=(their S6 rows), w, names) -- see render -- and None
    elsewhere, plus this rank's counts.  names (the rank's pair names, optional: render needs
    them) are sent to rank 0 for the reads the products name (S4's tmp1 reads, the survivors)
    over host_group; s4_reads: rank 0 also collects S4's reads (render's SAM text needs them)."""
    import torch

    from .blat import MAX_ROWS
    from .genome import MAX_REC, REC_DTYPE
    from .shard import shard_pairs
    dev = torch.device(device)
    L = backend.local_phase()
    g0 = 2 * int(lo)
    s5 = L.s5
    k5, r5 = _t(s5["key"], dev, torch.int64), _t(s5["row"], dev, torch.int64) + g0
    n5 = int(k5.numel())
    # S5's global order: every split read's ordinal (its bwa read id) and QNAME-group flag
    K5 = _allgatherv(torch.stack([k5, r5], 1), group, world)
    o5 = _order(K5[:, 0], K5[:, 1])
    ordinal = torch.empty_like(o5)
    ordinal[o5] = torch.arange(o5.numel(), device=dev)
    n_rank = _allgatherv(torch.tensor([[n5]], dtype=torch.int64, device=dev), group, world)[:, 0]
    base = int(n_rank[:rank].sum())
    ids = ordinal[base:base + n5].contiguous()
    cont = torch.zeros(n5, dtype=torch.uint8, device=dev)
    p5, nc5 = _t(s5["pos"], dev, torch.int64), _t(s5["ncig"], dev, torch.int64)
    c5 = _t(s5["cigar"], dev).view(torch.int32) if n5 else torch.zeros((0, 32), dtype=torch.int32, device=dev)
    has = torch.nonzero(ids > 0).reshape(-1)
    if has.numel():
        # the global predecessor of each query, when it is one of ours: the same QNAME (pair,
        # POS, CIGAR) continues its group
        pred = K5[o5[ids[has] - 1], 1]
        srt = torch.argsort(r5)
        rs = r5[srt]
        at = torch.searchsorted(rs, pred).clamp_(max=n5 - 1)
        mine = rs[at] == pred
        i, j = has[mine], srt[at[mine]]
        live = torch.arange(c5.shape[1], device=dev)[None, :] < nc5[i][:, None]
        same = (r5[j] // 2 == r5[i] // 2) & (p5[j] == p5[i]) & (nc5[j] == nc5[i]) & \
            ((c5[j] == c5[i]) | ~live).all(dim=1)
        cont[i] = same.to(torch.uint8)
    surv = backend.s5_s6_phase(ids, cont)
    # the survivors (ordinal, POS, CIGAR, S5 SEQ, S6 query) and their S6 rows, to rank 0
    src = _t(surv["src"], dev, torch.int64)
    ns = int(src.numel())
    l5 = _t(s5["len"], dev, torch.int64)
    l6 = _t(surv["s6_len"], dev, torch.int64)
    npsl = _t(surv["n_psl"], dev, torch.int64)
    W = _allgatherv(torch.tensor([[_width(l5), _width(l6)]], dtype=torch.int64, device=dev), group, world)
    w5, w6 = (int(v) for v in W.max(dim=0).values)
    s5b = _block(_t(s5["seq"], dev, torch.uint8), l5, src, w5)
    s6b = _block(_t(surv["s6_seq"], dev, torch.uint8), l6, torch.arange(ns, device=dev), w6)
    ords = ids[src]
    rows = torch.cat([_words(ords), _words(p5[src].to(torch.int32)), _words(nc5[src].to(torch.int32)), c5[src],
                      _words(l5[src].to(torch.int32)), _words(l6.to(torch.int32)), _words(npsl.to(torch.int32)),
                      _words(s5b), _words(s6b), _words(r5[src])], dim=1)  # the read's global row: render's names
    P6 = _t(surv["psl"], dev).view(torch.int32).reshape(ns, MAX_ROWS, PSL_WORDS)
    kk, rr = torch.nonzero(torch.arange(P6.shape[1], device=dev)[None, :] < npsl[:, None], as_tuple=True)
    table = torch.cat([_words(ords[kk]), P6[kk, rr]], dim=1)
    # the rows past MAX_ROWS (the backend's spill pool), tagged with their query's ordinal
    sq = _t(surv["spill_q"], dev, torch.int64) if "spill_q" in surv else torch.zeros(0, dtype=torch.int64, device=dev)
    SP = _t(surv["spill_psl"], dev).view(torch.int32).reshape(-1, PSL_WORDS) if "spill_psl" in surv else \
        torch.zeros((0, PSL_WORDS), dtype=torch.int32, device=dev)
    sp_table = torch.cat([_words(ords[sq]), SP], dim=1)
    all_rows = _gatherv(rows, group, world, rank)
    all_psl = _gatherv(table, group, world, rank)
    all_spill = _gatherv(sp_table, group, world, rank)
    # S4's stream: tmp1 / tmp2 of every rank zipped in the global order, from their keys alone
    t1, t2 = L.t1, L.t2
    k1, r1, l1 = _t(t1["key"], dev, torch.int64), _t(t1["row"], dev, torch.int64) + g0, _t(t1["len"], dev, torch.int64)
    k2, r2, l2 = _t(t2["key"], dev, torch.int64), _t(t2["row"], dev, torch.int64) + g0, _t(t2["len"], dev, torch.int64)
    M1 = _allgatherv(torch.stack([k1, r1, l1], 1), group, world)
    M2 = _allgatherv(torch.stack([k2, r2, l2], 1), group, world)
    z1, z2 = _order(M1[:, 0], M1[:, 1]), _order(M2[:, 0], M2[:, 1])
    n_pair = min(int(z1.numel()), int(z2.numel()))
    g1, g2 = M1[z1[:n_pair], 1], M2[z2[:n_pair], 1]
    ql = torch.stack([M1[z1[:n_pair], 2], M2[z2[:n_pair], 2]], 1).reshape(-1)
    W4 = _width(ql)
    counts = dict(tmp1=int(k1.numel()), tmp2=int(k2.numel()), s5_split_reads=n5, s6_queries=ns, s4_pairs=n_pair)
    recs = nrec = q_all = None
    if n_pair:
        bases = ql.reshape(-1, 2).sum(dim=1).cpu().numpy()
        shares = [shard_pairs(bases, d, world, backend.chunk_bases) for d in range(world)]
        starts = _allgatherv(torch.tensor([[g0]], dtype=torch.int64, device=dev), group, world)[:, 0]
        q_mine = _s4_reads(t1, t2, r1, r2, g1, g2, shares, starts, W4, rank, world, group, dev)
        a, b = shares[rank]
        words = REC_DTYPE.itemsize // 4
        if b > a:
            rw, rn = backend.s4_phase(q_mine, ql[2 * a:2 * b].to(torch.int32), pair_base=a)
            rw = _t(rw, dev).view(torch.int32).reshape(2 * (b - a), MAX_REC, words)
            rn = _t(rn, dev, torch.int64).clamp(max=MAX_REC)
            rr4, kk4 = torch.nonzero(torch.arange(MAX_REC, device=dev)[None, :] < rn[:, None], as_tuple=True)
            comp = torch.cat([_words(rr4 + 2 * a), _words(kk4.to(torch.int32)), rw[rr4, kk4]], dim=1)
        else:
            rn = torch.zeros(0, dtype=torch.int64, device=dev)
            comp = torch.zeros((0, 3 + words), dtype=torch.int32, device=dev)
        comp = _gatherv(comp, group, world, rank)
        cnt = _gatherv(rn.to(torch.int32).reshape(-1, 1), group, world, rank)
        qa = _gatherv(q_mine, group, world, rank) if s4_reads else None
        if rank == 0:
            recs = torch.zeros((2 * n_pair, MAX_REC, words), dtype=torch.int32, device=dev)
            recs[_i64(comp[:, :2]), comp[:, 2].long()] = comp[:, 3:]
            nrec, q_all = cnt.reshape(-1), qa
    named = None
    if names is not None:
        want = np.concatenate([r1.cpu().numpy(), r5[src].cpu().numpy()]) - g0
        mine = {int(r) + g0: names[int(r) // 2] for r in want}
        if world > 1:  # only rank 0 renders: the names go there alone
            import torch.distributed as dist
            parts = [None] * world if rank == 0 else None
            dist.gather_object(mine, parts, dst=0, group=host_group)
            named = {k: v for p in parts for k, v in p.items()} if rank == 0 else None
        else:
            named = mine
    if rank != 0:
        return None, counts
    order = torch.argsort(_i64(all_rows[:, :2]), stable=True)
    porder = torch.argsort(_i64(all_psl[:, :2]), stable=True)
    return dict(s4=(q_all, ql, recs, nrec, g1), surv=all_rows[order], psl=all_psl[porder], w=(w5, w6), names=named,
                max_rows=MAX_ROWS, spill=all_spill), counts


def _s4_reads(t1, t2, r1, r2, g1, g2, shares, starts, W4, rank, world, group, dev):
    """The reads of this rank's S4 share (pair-major uint8 [2 (b - a), W4]), each sent by the rank
    that holds it: for every destination d and its zipped pairs k in shares[d], the tmp1 read
    g1[k] and the tmp2 read g2[k] go from their owners (the rank whose rows start at or below
    them) -- one all-to-all per list, in k order."""
    import torch
    owner1 = torch.searchsorted(starts, g1, right=True) - 1
    owner2 = torch.searchsorted(starts, g2, right=True) - 1
    a, b = shares[rank]
    q = torch.full((2 * (b - a), W4), ord("N"), dtype=torch.uint8, device=dev)
    for t, r_own, g, owner, mate in ((t1, r1, g1, owner1, 0), (t2, r2, g2, owner2, 1)):
        seq = _t(t["seq"], dev, torch.uint8) if r_own.numel() else torch.zeros((0, 1), dtype=torch.uint8, device=dev)
        lens = _t(t["len"], dev, torch.int64)
        srt = torch.argsort(r_own)
        parts, recv = [], []
        for d in range(world):
            da, db = shares[d]
            ks = torch.arange(da, db, device=dev)
            sent = ks[owner[da:db] == rank]                 # pairs of d whose read this rank holds
            idx = srt[torch.searchsorted(r_own[srt], g[sent])] if sent.numel() else sent
            parts.append(_block(seq, lens, idx, W4))
        for s in range(world):
            recv.append(int((owner[a:b] == s).sum()))
        got = _alltoallv(parts, recv, group, world)
        # the rows from source s are this share's pairs owned by s, in k order
        ks = torch.arange(a, b, device=dev)
        pos = torch.cat([ks[owner[a:b] == s] for s in range(world)]) - a
        q[2 * pos + mate] = got
    return q


def render(result, backend, gene, genome_names, s4_text=True):
    """What consume_products reads, from search's rank-0 result (searched with names, and with
    s4_reads for s4_text): S4's SAM lines (blocks.S4Records, the fields Find_blocks reads,
    without s4_text), the split_sam lines of the survivors (split.fa order) and S6's PSL."""
    from .blat import PSL_DTYPE, spilled_rows
    from .blocks import S4Records
    from .genome import REC_DTYPE
    q, ql, recs, nrec, g1 = result["s4"]
    g1 = g1.cpu().numpy()
    named = result["names"]
    pn = [named[int(g)] for g in g1]
    if recs is not None:
        recs = recs.cpu().numpy().view(REC_DTYPE).reshape(recs.shape[0], recs.shape[1])
        nrec = nrec.cpu().numpy()
    else:
        nrec = np.zeros(0, np.int32)
    if not s4_text:
        s4 = S4Records(pn, recs, nrec, genome_names)
    else:
        s4 = []
        if len(g1):
            q, ql = q.cpu().numpy(), ql.cpu().numpy()
            for k in range(len(g1)):
                for m in (0, 1):
                    r = 2 * k + m
                    s4 += sam_lines(genome_names, pn[k], q[r, :ql[r]].tobytes().decode(), recs[r], nrec[r])
    S = result["surv"].cpu().numpy()
    w5, w6 = result["w"]
    n = S.shape[0]
    split_sam, psl = [], []
    if n:
        pos, ncig = S[:, 2], S[:, 3]
        cig = S[:, 4:36].copy().view(np.uint32)
        l5, l6, npsl = S[:, 36], S[:, 37], S[:, 38]
        s5 = S[:, 39:39 + w5 // 4].copy().view(np.uint8).reshape(n, w5)
        s6 = S[:, 39 + w5 // 4:39 + (w5 + w6) // 4].copy().view(np.uint8).reshape(n, w6)
        grow = S[:, 39 + (w5 + w6) // 4:].copy().view(np.int64).reshape(-1)
        qn = [named[int(g)] for g in grow]
        for k in range(n):
            split_sam.append(f"{qn[k]}\t0\t{gene}\t{int(pos[k]) + 1}\t60\t{cigar_string(cig[k], ncig[k])}\t=\t1111\t0\t"
                             f"{s5[k, :l5[k]].tobytes().decode()}\tA\n")
        table = result["psl"].cpu().numpy()
        rows = np.zeros((n, result["max_rows"]), PSL_DTYPE)
        r = 0
        for k in range(n):
            m = max(0, int(npsl[k]))
            if m:
                rows[k, :m] = table[r:r + m, 2:].copy().view(PSL_DTYPE).reshape(m)
            r += m
        extra = {}
        sp = result.get("spill")
        if sp is not None and len(sp):
            sp = sp.cpu().numpy()
            at = {int(o): k for k, o in enumerate(S[:, :2].copy().view(np.int64).reshape(-1))}
            qk = np.array([at[int(o)] for o in sp[:, :2].copy().view(np.int64).reshape(-1)], np.int64)
            extra = spilled_rows(sp[:, 2:].copy().view(PSL_DTYPE).reshape(-1), qk)
        psl = PSL_HEADER + backend.psl_lines([(str(k), s6[k, :l6[k]].tobytes().decode()) for k in range(n)], rows,
                                             npsl, extra=extra)
    return s4, split_sam, psl
