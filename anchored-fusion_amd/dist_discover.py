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
`af_s5_filter_device` with d_cont); S4 runs over the globally zipped pairs (all-gathered), each
rank on its share of that stream's bwa chunks, the records gathered to rank 0.  Rank 0 gathers the survivors and their S6 rows and orders them by
ordinal.  `search` stops there (the bench step); `render` turns the result into the texts
`pipeline.consume_products` reads, equal to the one-process run's byte for byte
(tests/test_dist_discover.py).

The per-rank work is done by a backend with three phases -- `local_phase` (S2 + S3 + the
gathers), `s4_phase(q, ql, pair_base)` (whole chunks of S4's stream) and `s5_s6_phase` -- implemented by discover.CandidateDiscovery
on the GPU; the tests run the CPU oracle through the same driver.  Every exchange is a tensor
all-gatherv (counts, then one max-padded all_gather) on `device` over `group`: RCCL on GPUs,
gloo on CPU; read names (for `render` only) go over `host_group` as objects.
"""
import numpy as np

from .genome import sam_lines

PSL_HEADER = ["psLayout version 3\n", "\n"]
_OPS = "MIDNSHP=X"


def cigar_string(words, n):
    return "".join(f"{int(v) >> 4}{_OPS[int(v) & 15]}" for v in words[:int(n)])


class LocalQueries:
    """A rank's lists after S2 + S3 + the gathers (host arrays; rows are local read rows).

    t1 / t2: the tmp1 / tmp2 rows in samtools order with their keys (2 pos + strand) and the reads
    as sequenced (seq uint8 [k, w], len int32 [k]: bytes past a row's length are ignored); s5: the
    split reads (the S5 queries) in order with keys, the anchored record's POS and CIGAR (cigar
    uint32 [k, 32], ncig), and the queries' SEQ in SAM orientation (seq uint8 [k, w], len).

    A backend's s5_s6_phase(ids, cont) returns dict(src int64 [m]: the survivors' S5 indices,
    s6_seq uint8 [m, w] + s6_len int32 [m]: their S6 queries, psl PSL_DTYPE [m, MAX_ROWS] +
    n_psl int32 [m]: their S6 rows)."""

    def __init__(self, t1, t2, s5):
        self.t1, self.t2, self.s5 = t1, t2, s5


def merge_order(keys, rows):
    """The global order of concatenated per-rank lists: by key, ties by global row."""
    return np.lexsort((np.asarray(rows, np.int64), np.asarray(keys, np.int64)))


def _allgatherv(arr, group, device, world):
    """All-gatherv of a 2-D numpy array (rows) over `group` on `device`; the rows of every rank
    in rank order (numpy).  world == 1: the array itself (no process group needed)."""
    import torch
    from .shard import allgatherv_device
    a = np.ascontiguousarray(arr)
    if world == 1:
        return a
    width = a.dtype.itemsize * int(np.prod(a.shape[1:]))
    t = torch.from_numpy(a.view(np.uint8).reshape(a.shape[0], width)).to(device)
    return allgatherv_device(t, group).cpu().numpy().view(a.dtype).reshape(-1, *a.shape[1:])


def _block(seq, lens, idx, width):
    """Rows idx of seq (uint8 [k, w]) as uint8 [len(idx), width], 'N' past each row's length."""
    idx = np.asarray(idx, np.int64)
    out = np.full((len(idx), width), ord("N"), np.uint8)
    if len(idx):
        w = min(width, int(seq.shape[1]))
        out[:, :w] = np.asarray(seq)[idx, :w]
        out[np.arange(width)[None, :] >= np.asarray(lens, np.int64)[idx][:, None]] = ord("N")
    return out


def _width(lens):
    """Row width for sequences of these lengths: the longest, at least 1, a multiple of 4."""
    w = max(1, int(np.max(lens)) if len(lens) else 1)
    return -(-w // 4) * 4


def _i32(a):
    return np.asarray(a, np.int64).astype(np.int32).reshape(-1, 1)


PSL_WORDS = 82  # af_psl / blat.PSL_DTYPE as int32 words (328 B)


def psl_table(surv, ords):
    """S6's rows of the survivors as int32 rows: ordinal (2 words) + one af_psl row, survivor by
    survivor, each one's rows in order."""
    from .blat import PSL_DTYPE
    n_psl = np.asarray(surv["n_psl"], np.int64)
    if not len(n_psl):
        return np.zeros((0, 2 + PSL_WORDS), np.int32)
    P = np.asarray(surv["psl"]).view(PSL_DTYPE).reshape(len(n_psl), -1)
    kk, rr = np.nonzero(np.arange(P.shape[1])[None, :] < n_psl[:, None])
    m = len(kk)
    sel = np.ascontiguousarray(P[kk, rr])
    return np.concatenate([np.asarray(ords, np.int64)[kk].view(np.int32).reshape(m, 2),
                           sel.view(np.int32).reshape(m, PSL_WORDS)], axis=1)


def psl_rows(table, n, npsl):
    """table (ordinal-sorted psl_table rows of n survivors) -> per survivor a PSL_DTYPE array of
    MAX_ROWS rows (the first npsl[k] valid)."""
    from .blat import MAX_ROWS, PSL_DTYPE
    out = np.zeros((n, MAX_ROWS), PSL_DTYPE)
    r = 0
    for k in range(n):
        m = max(0, int(npsl[k]))
        if m:
            out[k, :m] = table[r:r + m, 2:].copy().view(PSL_DTYPE).reshape(m)
        r += m
    return out


def _s4_sharded(backend, q, ql, rank, world, group, device):
    """S4 over the zipped pairs q / ql (every rank holds them): this rank aligns its share of the
    stream's bwa chunks (shard.shard_pairs over the pairs' bases, pair_base = its first pair);
    the records (compacted: one row per printed record, with its read and slot) are gathered
    and rank 0 returns (recs REC_DTYPE [2 P, MAX_REC], nrec [2 P]); other ranks (None, None)."""
    from .genome import MAX_REC, REC_DTYPE
    from .shard import shard_pairs
    P = len(ql) // 2
    if not P:
        return None, np.zeros(0, np.int32)
    lo, hi = shard_pairs(ql.astype(np.int64).reshape(-1, 2).sum(axis=1), rank, world, backend.chunk_bases)
    words = REC_DTYPE.itemsize // 4
    if hi > lo:
        r, n = backend.s4_phase(q[2 * lo:2 * hi], ql[2 * lo:2 * hi], pair_base=lo)
        n = np.minimum(np.asarray(n, np.int64), MAX_REC)
        rr, kk = np.nonzero(np.arange(MAX_REC)[None, :] < n[:, None])
        body = np.ascontiguousarray(r[rr, kk]).view(np.int32).reshape(len(rr), words)
        rows = np.concatenate([(rr + 2 * lo).astype(np.int64).view(np.int32).reshape(-1, 2),
                               kk.astype(np.int32).reshape(-1, 1), body], axis=1)
        cnt = n.astype(np.int32).reshape(-1, 1)
    else:
        rows = np.zeros((0, 3 + words), np.int32)
        cnt = np.zeros((0, 1), np.int32)
    rows = _allgatherv(rows, group, device, world)
    cnt = _allgatherv(cnt, group, device, world)[:, 0]
    if rank != 0:
        return None, None
    recs = np.zeros((2 * P, MAX_REC), REC_DTYPE)
    read = rows[:, :2].copy().view(np.int64).reshape(-1)
    recs[read, rows[:, 2]] = np.ascontiguousarray(rows[:, 3:]).view(REC_DTYPE).reshape(-1)
    return recs, cnt


def search(backend, lo, rank, world, group=None, device="cpu", names=None, host_group=None):
    """The distributed S3-S6 of one gene (backend already holds this rank's S2 input).  Returns,
    on rank 0, dict(s4=(pair reads, lens, records, counts, t1 global rows), surv=(ordinal-sorted
    survivor rows), psl=(their S6 rows), names=...) -- see render -- and None elsewhere, plus this
    rank's counts.  names (the rank's pair names, optional: render needs them) are sent to rank 0
    for the reads the texts name (S4's tmp1 reads, the survivors) over host_group."""
    L = backend.local_phase()
    g0 = 2 * int(lo)

    def kr(d):
        return np.stack([np.asarray(d["key"], np.int64), np.asarray(d["row"], np.int64) + g0], axis=1) \
            if len(d["key"]) else np.zeros((0, 2), np.int64)
    # the lists' keys, every rank (S5 ids and groups; S4's global zip on rank 0)
    K5 = _allgatherv(kr(L.s5), group, device, world)
    n_before = _allgatherv(np.array([[len(L.s5["key"])]], np.int64), group, device, world)[:, 0]
    o5 = merge_order(K5[:, 0], K5[:, 1])
    ordinal = np.empty(len(o5), np.int64)
    ordinal[o5] = np.arange(len(o5))
    base = int(n_before[:rank].sum())
    n5 = len(L.s5["key"])
    ids = ordinal[base:base + n5]
    cont = np.zeros(n5, np.uint8)
    rows5 = np.asarray(L.s5["row"], np.int64) + g0
    has = np.nonzero(ids > 0)[0]
    if len(has):
        # the global predecessor of each query, when it is one of ours: then the same QNAME
        # (pair, POS, CIGAR) continues its group
        pred = K5[o5[ids[has] - 1], 1]
        srt = np.argsort(rows5, kind="stable")
        at = np.minimum(np.searchsorted(rows5[srt], pred), n5 - 1)
        mine = rows5[srt][at] == pred
        i, j = has[mine], srt[at][mine]
        r5, p5, nc5 = (np.asarray(L.s5[k], np.int64) for k in ("row", "pos", "ncig"))
        c5 = np.asarray(L.s5["cigar"], np.uint32)
        live = np.arange(c5.shape[1])[None, :] < nc5[i][:, None]
        same = (r5[j] // 2 == r5[i] // 2) & (p5[j] == p5[i]) & (nc5[j] == nc5[i]) & \
            ((c5[j] == c5[i]) | ~live).all(axis=1)
        cont[i] = same
    surv = backend.s5_s6_phase(ids, cont)
    # the survivors (ordinal, POS, CIGAR, S5 SEQ, S6 query) and their S6 rows, to every rank
    src = np.asarray(surv["src"], np.int64)
    ns = len(src)
    l5 = np.asarray(L.s5["len"], np.int64)
    l6 = np.asarray(surv["s6_len"], np.int64)
    W5 = _allgatherv(np.array([[_width(l5), _width(l6)]], np.int64), group, device, world).max(axis=0)
    s5b = _block(L.s5["seq"], l5, src, int(W5[0]))
    s6b = _block(surv["s6_seq"], l6, np.arange(ns), int(W5[1]))
    ords = ids[src] if ns else np.zeros(0, np.int64)
    cig = np.asarray(L.s5["cigar"], np.uint32)[src] if ns else np.zeros((0, 32), np.uint32)
    rows = np.concatenate([
        ords.astype(np.int64).view(np.int32).reshape(-1, 2),
        _i32(np.asarray(L.s5["pos"])[src] if ns else []), _i32(np.asarray(L.s5["ncig"])[src] if ns else []),
        cig.view(np.int32).reshape(-1, 32), _i32(l5[src]), _i32(l6), _i32(surv["n_psl"]),
        s5b.view(np.int32).reshape(ns, int(W5[0]) // 4), s6b.view(np.int32).reshape(ns, int(W5[1]) // 4),
        # the read's global row (render: names)
        (rows5[src] if ns else np.zeros(0, np.int64)).view(np.int32).reshape(-1, 2)], axis=1)
    psl = psl_table(surv, ords)
    all_rows = _allgatherv(rows.astype(np.int32), group, device, world)
    all_psl = _allgatherv(psl, group, device, world)
    # S4's reads: the rank's tmp1 / tmp2 reads with their keys and global rows
    W4 = int(_allgatherv(np.array([[_width(np.concatenate([np.asarray(L.t1["len"], np.int64),
                                                            np.asarray(L.t2["len"], np.int64)]))]], np.int64),
                         group, device, world).max())

    def reads_rows(d):
        k = len(d["key"])
        if not k:
            return np.zeros((0, 5 + W4 // 4), np.int32)
        return np.concatenate([np.stack([np.asarray(d["key"], np.int64), np.asarray(d["row"], np.int64) + g0],
                                        axis=1).view(np.int32).reshape(k, 4), _i32(d["len"]),
                               _block(d["seq"], d["len"], np.arange(k), W4).view(np.int32).reshape(k, W4 // 4)],
                              axis=1)
    T1 = _allgatherv(reads_rows(L.t1), group, device, world)
    T2 = _allgatherv(reads_rows(L.t2), group, device, world)
    counts = dict(tmp1=len(L.t1["key"]), tmp2=len(L.t2["key"]), s5_split_reads=n5, s6_queries=ns)
    named = None
    if names is not None:
        want = list(np.asarray(L.t1["row"], np.int64)) + [int(r) - g0 for r in (rows5[src] if ns else [])]
        mine = {int(r) + g0: names[int(r) // 2] for r in want}
        if world > 1:
            import torch.distributed as dist
            parts = [None] * world
            dist.all_gather_object(parts, mine, group=host_group)
            named = {k: v for p in parts for k, v in p.items()}
        else:
            named = mine
    def split_reads(T):
        kg = T[:, :4].copy().view(np.int64).reshape(-1, 2)
        o = merge_order(kg[:, 0], kg[:, 1])
        seq = T[o, 5:].copy().view(np.uint8).reshape(len(o), -1)
        return kg[o, 1], T[o, 4], seq
    # S4's input stream (tmp1 / tmp2 zipped in samtools order), the same on every rank; each rank
    # aligns whole bwa chunks of it (its read ids and insert-size chunks those of one run) and
    # rank 0 collects the records
    g1, l1, q1 = split_reads(T1)
    g2, l2, q2 = split_reads(T2)
    n_pair = min(len(g1), len(g2))
    q = np.full((2 * n_pair, W4), ord("N"), np.uint8)
    ql = np.zeros(2 * n_pair, np.int32)
    if n_pair:
        q[0::2], q[1::2] = q1[:n_pair], q2[:n_pair]
        ql[0::2], ql[1::2] = l1[:n_pair], l2[:n_pair]
    recs, nrec = _s4_sharded(backend, q, ql, rank, world, group, device)
    counts["s4_pairs"] = n_pair
    if rank != 0:
        return None, counts
    order = np.argsort(all_rows[:, :2].copy().view(np.int64).reshape(-1), kind="stable")
    pk = all_psl[:, :2].copy().view(np.int64).reshape(-1)
    porder = np.argsort(pk, kind="stable")
    return dict(s4=(q, ql, recs, nrec, g1[:n_pair]), surv=all_rows[order], psl=all_psl[porder],
                w=(int(W5[0]), int(W5[1])), names=named), counts


def render(result, backend, gene, genome_names, s4_text=True):
    """What consume_products reads, from search's rank-0 result (searched with names): S4's SAM
    lines (blocks.S4Records, the fields Find_blocks reads, without s4_text), the split_sam lines
    of the survivors (split.fa order) and S6's PSL."""
    from .blocks import S4Records
    q, ql, recs, nrec, g1 = result["s4"]
    named = result["names"]
    s4 = []
    pn = [named[int(g)] for g in g1]
    if not s4_text:
        s4 = S4Records(pn, recs if len(g1) else None, nrec, genome_names)
    elif len(g1):
        for k in range(len(g1)):
            sa = q[2 * k, :ql[2 * k]].tobytes().decode()
            sb = q[2 * k + 1, :ql[2 * k + 1]].tobytes().decode()
            s4 += sam_lines(genome_names, pn[k], sa, recs[2 * k], nrec[2 * k])
            s4 += sam_lines(genome_names, pn[k], sb, recs[2 * k + 1], nrec[2 * k + 1])
    S = result["surv"]
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
        rows = psl_rows(result["psl"], n, npsl)
        psl = PSL_HEADER + backend.psl_lines([(str(k), s6[k, :l6[k]].tobytes().decode()) for k in range(n)], rows,
                                             npsl)
    return s4, split_sam, psl
