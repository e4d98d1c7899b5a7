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
QNAME (then both are the same pair's mates, on the same rank).  S5, its check and S6 then run on
every rank over its own queries with those ids and group flags (`af_genome_align_se_ids_device`,
`af_s5_filter_device` with d_cont); S4 runs on rank 0 over the globally zipped pairs, whose reads
the ranks send there.  Rank 0 gathers the survivors and their S6 rows, orders them by ordinal
and returns the texts `pipeline.consume_products` reads.  The result is the one-process run's,
byte for byte (tests/test_dist_discover.py).

The per-rank work is done by a backend with three phases -- `local_phase` (S2 + S3 + the
gathers), `s4_phase` (rank 0) and `s5_s6_phase` -- implemented by discover.CandidateDiscovery
on the GPU; the tests also run the CPU oracle through the same driver.  Host data moves over
`host_group`, a CPU (gloo) group.
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
    as sequenced (seqs [k, w], lens); s5: the split reads (the S5 queries) in order with keys, the
    anchored record's POS and CIGAR (words, n), and the queries' SEQ in SAM orientation."""

    def __init__(self, t1, t2, s5):
        self.t1, self.t2, self.s5 = t1, t2, s5


def merge_order(keys, rows):
    """The global order of concatenated per-rank lists: by key, ties by global row."""
    return np.lexsort((np.asarray(rows, np.int64), np.asarray(keys, np.int64)))


def _all_gather(obj, group):
    import torch.distributed as dist
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


def _gather0(obj, group):
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    out = [None] * world if rank == 0 else None
    dist.gather_object(obj, out, dst=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return out


def run(backend, lo, names, gene, genome_names, rank, world, host_group, log=print):
    """S3-S6 of one gene over the ranks (backend already holds this rank's S2 input).  names: the
    rank's pair names (local pair index).  Returns (s4 SAM lines, split_sam lines, S6 PSL lines)
    on rank 0, None elsewhere, plus this rank's step counts."""
    L = backend.local_phase()
    g0 = 2 * int(lo)
    mine = dict(t1=(L.t1["key"], L.t1["row"] + g0), t2=(L.t2["key"], L.t2["row"] + g0),
                s5=(L.s5["key"], L.s5["row"] + g0))
    every = _all_gather(mine, host_group) if world > 1 else [mine]
    # S5: global ordinals (bwa's read ids in split.fa) and QNAME groups
    k5 = np.concatenate([e["s5"][0] for e in every])
    r5 = np.concatenate([e["s5"][1] for e in every])
    o5 = merge_order(k5, r5)
    pos_of = np.empty(len(o5), np.int64)
    pos_of[o5] = np.arange(len(o5))
    base = sum(len(e["s5"][0]) for e in every[:rank])
    n5 = len(L.s5["key"])
    ids = pos_of[base:base + n5]
    prev = np.full(n5, -1, np.int64)  # the global predecessor, as a local index when it is ours
    loc_of = {int(r): i for i, r in enumerate(L.s5["row"] + g0)}
    for i in range(n5):
        if ids[i] > 0:
            prev[i] = loc_of.get(int(r5[o5[ids[i] - 1]]), -1)
    cont = np.zeros(n5, np.uint8)
    for i in range(n5):
        j = prev[i]
        if j >= 0:
            a, b = int(L.s5["row"][j]), int(L.s5["row"][i])
            cont[i] = a // 2 == b // 2 and L.s5["pos"][j] == L.s5["pos"][i] and \
                L.s5["ncig"][j] == L.s5["ncig"][i] and \
                np.array_equal(L.s5["cigar"][j, :L.s5["ncig"][j]], L.s5["cigar"][i, :L.s5["ncig"][i]])
    surv = backend.s5_s6_phase(ids, cont)
    # the survivors to rank 0: ordinal, QNAME line fields, the S6 query and its rows
    rows_out = []
    for k, src in enumerate(surv["src"]):
        src = int(src)
        r = int(L.s5["row"][src])
        rows_out.append((int(ids[src]), names[r // 2], int(L.s5["pos"][src]) + 1,
                         cigar_string(L.s5["cigar"][src], L.s5["ncig"][src]), L.s5["seq"][src], surv["s6_seq"][k],
                         surv["psl"][k], int(surv["n_psl"][k])))
    # S4's reads to rank 0: the rank's tmp1 / tmp2 reads (sequenced orientation) with their rows
    s4_mine = dict(t1=(L.t1["row"] + g0, L.t1["seq"], L.t1["len"], [names[int(r) // 2] for r in L.t1["row"]]),
                   t2=(L.t2["row"] + g0, L.t2["seq"], L.t2["len"]))
    got = _gather0((rows_out, s4_mine), host_group) if world > 1 else [(rows_out, s4_mine)]
    counts = dict(tmp1=len(L.t1["key"]), tmp2=len(L.t2["key"]), s5_split_reads=n5, s6_queries=len(surv["src"]))
    if rank != 0:
        return None, counts
    # S4 on rank 0 over the globally zipped lists
    k1 = np.concatenate([e["t1"][0] for e in every])
    r1 = np.concatenate([e["t1"][1] for e in every])
    k2 = np.concatenate([e["t2"][0] for e in every])
    r2 = np.concatenate([e["t2"][1] for e in every])
    o1, o2 = merge_order(k1, r1), merge_order(k2, r2)
    n_pair = min(len(o1), len(o2))
    seqs, lens, pname = {}, {}, {}
    for _, s4 in got:
        for rr, sq, ln, nm in zip(s4["t1"][0], s4["t1"][1], s4["t1"][2], s4["t1"][3]):
            seqs[int(rr)], lens[int(rr)], pname[int(rr)] = sq, int(ln), nm
        for rr, sq, ln in zip(s4["t2"][0], s4["t2"][1], s4["t2"][2]):
            seqs[int(rr)], lens[int(rr)] = sq, int(ln)
    s4_lines = []
    if n_pair:
        a_rows = [int(r1[o1[k]]) for k in range(n_pair)]
        b_rows = [int(r2[o2[k]]) for k in range(n_pair)]
        w = max(max(len(seqs[r]) for r in a_rows), max(len(seqs[r]) for r in b_rows))
        q = np.full((2 * n_pair, w), ord("N"), np.uint8)
        ql = np.empty(2 * n_pair, np.int32)
        for k, (a, b) in enumerate(zip(a_rows, b_rows)):
            q[2 * k, :len(seqs[a])], q[2 * k + 1, :len(seqs[b])] = seqs[a], seqs[b]
            ql[2 * k], ql[2 * k + 1] = lens[a], lens[b]
        recs, nrec = backend.s4_phase(q, ql)
        for k, a in enumerate(a_rows):
            sa = q[2 * k, :ql[2 * k]].tobytes().decode()
            sb = q[2 * k + 1, :ql[2 * k + 1]].tobytes().decode()
            s4_lines += sam_lines(genome_names, pname[a], sa, recs[2 * k], nrec[2 * k])
            s4_lines += sam_lines(genome_names, pname[a], sb, recs[2 * k + 1], nrec[2 * k + 1])
    # the survivors in split.fa order: split_sam lines and S6's PSL (ids = ordinals)
    surv_all = sorted((x for rows, _ in got for x in rows), key=lambda x: x[0])
    split_sam = [f"{nm}\t0\t{gene}\t{pos}\t60\t{cig}\t=\t1111\t0\t{seq}\tA\n"
                 for _, nm, pos, cig, seq, _, _, _ in surv_all]
    psl = []
    if surv_all:
        psl = PSL_HEADER + backend.psl_lines([(str(k), x[5]) for k, x in enumerate(surv_all)],
                                             [x[6] for x in surv_all], [x[7] for x in surv_all])
    counts["s4_pairs"] = n_pair
    return (s4_lines, split_sam, psl), counts
