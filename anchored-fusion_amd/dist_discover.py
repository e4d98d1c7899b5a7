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
`af_s5_filter_device` with d_cont); S4 runs on rank 0 over the globally zipped pairs, whose reads
the ranks send there.  Rank 0 gathers the survivors and their S6 rows and orders them by
ordinal.  `search` stops there (the bench step); `render` turns the result into the texts
`pipeline.consume_products` reads, equal to the one-process run's byte for byte
(tests/test_dist_discover.py).

The per-rank work is done by a backend with three phases -- `local_phase` (S2 + S3 + the
gathers), `s4_phase` (rank 0) and `s5_s6_phase` -- implemented by discover.CandidateDiscovery
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
    as sequenced (seq uint8 [k, w], len); s5: the split reads (the S5 queries) in order with keys,
    the anchored record's POS and CIGAR (cigar uint32 [k, 32], ncig), and the queries' SEQ in SAM
    orientation (seq uint8 [k, w], len)."""

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


def _pad_rows(rows, w):
    out = np.full((len(rows), w), ord("N"), np.uint8)
    for i, r in enumerate(rows):
        out[i, :len(r)] = r
    return out


def _i32(a):
    return np.asarray(a, np.int64).astype(np.int32).reshape(-1, 1)


def _u8(x):
    """A sequence as uint8 (bytes, str or an array)."""
    if isinstance(x, str):
        return np.frombuffer(x.encode(), np.uint8)
    if isinstance(x, (bytes, bytearray)):
        return np.frombuffer(bytes(x), np.uint8)
    return np.asarray(x, np.uint8)


PSL_WORDS = 82  # af_psl / blat.PSL_DTYPE as int32 words (328 B)


def psl_table(surv, ords):
    """S6's rows of the survivors as int32 rows: ordinal (2 words) + one af_psl row."""
    from .blat import PSL_DTYPE
    parts = []
    for k, o in enumerate(ords):
        m = int(surv["n_psl"][k])
        if m <= 0:
            continue
        r = np.ascontiguousarray(np.asarray(surv["psl"][k])[:m]).view(PSL_DTYPE)
        parts.append(np.concatenate([np.full((m, 1), int(o), np.int64).view(np.int32).reshape(m, 2),
                                     r.view(np.int32).reshape(m, PSL_WORDS)], axis=1))
    return np.concatenate(parts) if parts else np.zeros((0, 2 + PSL_WORDS), np.int32)


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
    local_of = {int(r): i for i, r in enumerate(rows5)}
    for i in range(n5):
        if ids[i] == 0:
            continue
        j = local_of.get(int(K5[o5[ids[i] - 1], 1]), -1)  # the global predecessor, when it is ours
        if j < 0:
            continue
        a, b = int(L.s5["row"][j]), int(L.s5["row"][i])
        cont[i] = a // 2 == b // 2 and L.s5["pos"][j] == L.s5["pos"][i] and L.s5["ncig"][j] == L.s5["ncig"][i] and \
            np.array_equal(L.s5["cigar"][j, :L.s5["ncig"][j]], L.s5["cigar"][i, :L.s5["ncig"][i]])
    surv = backend.s5_s6_phase(ids, cont)
    # the survivors (ordinal, POS, CIGAR, S5 SEQ, S6 query) and their S6 rows, to every rank
    src = np.asarray(surv["src"], np.int64)
    ns = len(src)
    w5 = max(1, int(max((len(x) for x in L.s5["seq"]), default=1)))
    w6 = max(1, int(max((len(x) for x in surv["s6_seq"]), default=1)))
    w5, w6 = -(-w5 // 4) * 4, -(-w6 // 4) * 4
    s5b = _pad_rows([_u8(L.s5["seq"][int(k)]) for k in src], w5)
    s6b = _pad_rows([_u8(x) for x in surv["s6_seq"]], w6)
    W5 = _allgatherv(np.array([[w5, w6]], np.int64), group, device, world).max(axis=0)
    s5b = np.pad(s5b, ((0, 0), (0, int(W5[0]) - w5)), constant_values=ord("N"))
    s6b = np.pad(s6b, ((0, 0), (0, int(W5[1]) - w6)), constant_values=ord("N"))
    ords = ids[src] if ns else np.zeros(0, np.int64)
    cig = np.asarray(L.s5["cigar"], np.uint32)[src] if ns else np.zeros((0, 32), np.uint32)
    rows = np.concatenate([
        ords.astype(np.int64).view(np.int32).reshape(-1, 2) if ns else np.zeros((0, 2), np.int32),
        _i32(np.asarray(L.s5["pos"])[src] if ns else []), _i32(np.asarray(L.s5["ncig"])[src] if ns else []),
        cig.view(np.int32).reshape(-1, 32),
        _i32([len(L.s5["seq"][int(k)]) for k in src]), _i32([len(x) for x in surv["s6_seq"]]),
        _i32(surv["n_psl"]), s5b.view(np.int32).reshape(ns, int(W5[0]) // 4),
        s6b.view(np.int32).reshape(ns, int(W5[1]) // 4),
        # the read's global row (render: names)
        (rows5[src] if ns else np.zeros(0, np.int64)).view(np.int32).reshape(-1, 2)], axis=1)
    psl = psl_table(surv, ords)
    all_rows = _allgatherv(rows.astype(np.int32), group, device, world)
    all_psl = _allgatherv(psl, group, device, world)
    # S4's reads: the rank's tmp1 / tmp2 reads with their keys and global rows
    w4 = max(1, int(max((len(_u8(x)) for x in list(L.t1["seq"]) + list(L.t2["seq"])), default=1)))
    W4 = int(_allgatherv(np.array([[w4]], np.int64), group, device, world).max())
    W4 = -(-W4 // 4) * 4

    def reads_rows(d):
        k = len(d["key"])
        if not k:
            return np.zeros((0, 5 + W4 // 4), np.int32)
        return np.concatenate([np.stack([np.asarray(d["key"], np.int64), np.asarray(d["row"], np.int64) + g0],
                                        axis=1).view(np.int32).reshape(k, 4), _i32(d["len"]),
                               _pad_rows([_u8(x) for x in d["seq"]], W4).view(np.int32).reshape(k, W4 // 4)], axis=1)
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
    if rank != 0:
        return None, counts

    def split_reads(T):
        kg = T[:, :4].copy().view(np.int64).reshape(-1, 2)
        o = merge_order(kg[:, 0], kg[:, 1])
        seq = T[o, 5:].copy().view(np.uint8).reshape(len(o), -1)
        return kg[o, 1], T[o, 4], seq
    g1, l1, q1 = split_reads(T1)
    g2, l2, q2 = split_reads(T2)
    n_pair = min(len(g1), len(g2))
    q = np.full((2 * n_pair, W4), ord("N"), np.uint8)
    ql = np.zeros(2 * n_pair, np.int32)
    if n_pair:
        q[0::2], q[1::2] = q1[:n_pair], q2[:n_pair]
        ql[0::2], ql[1::2] = l1[:n_pair], l2[:n_pair]
        recs, nrec = backend.s4_phase(q, ql)
    else:
        recs, nrec = None, np.zeros(0, np.int32)
    order = np.argsort(all_rows[:, :2].copy().view(np.int64).reshape(-1), kind="stable")
    pk = all_psl[:, :2].copy().view(np.int64).reshape(-1)
    porder = np.argsort(pk, kind="stable")
    counts["s4_pairs"] = n_pair
    return dict(s4=(q, ql, recs, nrec, g1[:n_pair]), surv=all_rows[order], psl=all_psl[porder],
                w=(int(W5[0]), int(W5[1])), names=named), counts


def render(result, backend, gene, genome_names):
    """The texts consume_products reads, from search's rank-0 result (searched with names): S4's
    SAM lines, the split_sam lines of the survivors (split.fa order) and S6's PSL."""
    q, ql, recs, nrec, g1 = result["s4"]
    named = result["names"]
    s4 = []
    if len(g1):
        pn = [named[int(g)] for g in g1]
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
