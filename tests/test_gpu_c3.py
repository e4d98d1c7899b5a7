"""configs[2] on the GPU: the device-made hg38-scale world (simworld) and the device pipeline
(discover.CandidateDiscovery: S2 + S3 + the S4/S5/S6 genome searches).

At full size (50 M pairs, 3.09 Gbp) the results are checked through properties (the bwa index
by fm_checks on samples, exact reads beyond 2^31 placed on their bases); the first bwa chunks of
the same pairs are checked bit-exactly against the CPU oracle (the GPU aligned them in the same
place of the same input stream, so read ids and insert-size chunks agree).  On the 2 % world
(62 Mbp) the bwa index and every S4 / S5 record equal the oracle's own index and genome calls."""
import numpy as np
import pytest

import oracle
from helpers import assert_records_equal

pytestmark = pytest.mark.gpu


def _world(anchor, scale):
    from anchored_fusion_amd import simworld
    return simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=scale)


def test_world_is_deterministic_and_distinct(anchor):
    import torch
    W1, W2 = _world(anchor, 0.01), _world(anchor, 0.01)
    assert torch.equal(W1.blob, W2.blob)
    a = W1.simulate_pairs(20000, read_len=150, seed=3)
    b = W2.simulate_pairs(20000, read_len=150, seed=3)
    assert torch.equal(a, b)
    c = W1.simulate_pairs(20000, read_len=150, seed=3, pair_base=20000)
    assert not torch.equal(a, c)
    g = W1.blob.cpu().numpy()
    vals = set(np.unique(g).tolist())
    assert vals <= set(b"ACGTN")
    # the embedded genes are in the genome as exons
    for name, spans in W1.loci.items():
        seq = W1.anchor if name == "anchor" else W1.partners[int(name[7:])]
        got = b"".join(bytes(g[W1.offsets[W1.names.index(c)] + s:W1.offsets[W1.names.index(c)] + e])
                       for c, s, e in spans)
        assert got == seq
    # repeats: far more repeated 16-mers than a random sequence of the same size would hold
    # (~1e6^2 / 2 / 4^16 ~ 0.01 % of the 16-mers of 1 Mb of random sequence repeat)
    body = g[W1.offsets[0] + 20000:W1.offsets[0] + 1_020_000]
    codes = np.searchsorted(np.frombuffer(b"ACGT", np.uint8), body).clip(0, 3).astype(np.uint64)
    k = np.zeros(len(codes) - 15, np.uint64)
    for u in range(16):
        k = (k << np.uint64(2)) | codes[u:u + len(k)]
    _, cnt = np.unique(k, return_counts=True)
    assert (cnt[cnt > 1].sum()) / len(k) > 0.02


def test_discovery_matches_oracle_reduced(anchor):
    """A reduced world end to end: records, S3 lists and the S4/S5 queries vs the host rules."""
    import torch

    from anchored_fusion_amd import discover
    from anchored_fusion_amd.align import AlignResult, partition
    W = _world(anchor, 0.02)
    ref = W.genome_index()
    tiles = W.tiles()
    # the oracle's bwa index of the same contigs (62 Mbp): text and suffix array row for row
    contigs = [(nm, W.blob[o:o + ln].cpu().numpy().tobytes()) for nm, o, ln in zip(W.names, W.offsets, W.lens)]
    og = oracle.OracleGenome(contigs)
    assert og.l_pac == ref.l_pac and og.primary() == ref.primary()
    assert np.array_equal(og.text(), ref.text())
    bad = np.nonzero(og.sa() != ref.sa())[0]
    assert bad.size == 0, f"{bad.size} suffix-array rows differ, first {bad[:5]}"
    n = 140_000
    reads_t = W.simulate_pairs(n, read_len=150, seed=9)
    d = discover.CandidateDiscovery(anchor, ref, tiles, n, 150, device=0, inflight=3, batch_chunks=1)
    d.run(reads_t)
    torch.cuda.synchronize()
    reads = reads_t.cpu().numpy()
    got = {k: v.cpu().numpy() for k, v in d.out.items()}
    got["cigar"] = got["cigar"].view(np.uint32)
    ref_rec = oracle.OracleIndex(anchor).align_pairs(reads, threads=8)
    assert_records_equal(got, ref_rec, reads)
    res = AlignResult(got["flag"], got["pos"], got["score"], got["n_cigar"], got["cigar"], got["hits"])
    t1, t2, an = partition(res)
    c = d.counts
    assert (c["tmp1"], c["tmp2"], c["anchored"]) == (len(t1), len(t2), len(an))
    assert np.array_equal(d.s3[0][:len(t1)].cpu().numpy(), t1)
    assert np.array_equal(d.s3[2][:len(an)].cpu().numpy(), an)
    # S4 queries interleave tmp1 / tmp2 as sequenced; S5 = anchored split reads as SAM prints them
    from anchored_fusion_amd.cigar import normalize
    comp = bytes.maketrans(b"ACGTN", b"TGCAN")
    want = []
    for a, b in zip(t1, t2):
        want += [(int(a), reads[a].tobytes()), (int(b), reads[b].tobytes())]
    for r in an:
        cig = res.cigar_str(r)
        s = reads[r].tobytes()
        if len(normalize(cig, s.decode())[0]) == 2:
            want.append((int(r), s[::-1].translate(comp) if got["flag"][r] & 0x10 else s))
    nq = int(d.n_q.item())
    assert nq == len(want)
    q = d.q[:nq].cpu().numpy()
    rows = d.q_rows[:nq].cpu().numpy()
    for k, (r, s) in enumerate(want):
        assert rows[k] == r and q[k].tobytes() == s
    # S4 / S5 records (af_grec) of the device calls == oracle/bwa_pe.c's genome calls (FM mode) on
    # the same queries and contigs: S4 with the step's chunk grid, S5 with its read ids
    _check_genome_records_oracle(d, og, q, nq, c["s4_pairs"])
    # S5's genome check and the S6 queries == the host chain over the same records
    _check_s5_s6(d, ref, reads, got, an, c["s4_pairs"], nq)
    summ = d.summary()
    assert summ["s6_queries"] > 0 and summ["s6_placed"] > 0.5 * summ["s6_queries"]
    assert summ["queries_placed"] > 0.9 * nq and summ["genome_cap_overflow"] == 0
    d.close()
    ref.close()
    tiles.close()


def _check_genome_records(d, ref, q, nq, npair):
    from anchored_fusion_amd import _lib, discover, genome
    recs = d.q_recs[:nq * discover.MAX_REC * genome.REC_DTYPE.itemsize].cpu().numpy().view(genome.REC_DTYPE)
    recs = recs.reshape(nq, discover.MAX_REC)
    nrec = d.q_nh[:nq].cpu().numpy()
    lens = d.q_lens[:nq].cpu().numpy()
    pe = _lib.default_pe(chunk_bases=d.chunk_bases, pair_base=0)
    r4, n4 = ref.align_pe(q[:2 * npair], lens[:2 * npair], pe=pe)
    r5, n5 = ref.align_se(q[2 * npair:nq], lens[2 * npair:nq], pe=pe)
    want_r, want_n = np.concatenate([r4, r5]), np.concatenate([n4, n5])
    assert np.array_equal(nrec, want_n)
    assert (nrec >= 1).all()
    for r in range(nq):
        for k in range(min(int(nrec[r]), discover.MAX_REC)):
            a, b = recs[r, k], want_r[r, k]
            nc = int(a["n_cigar"])
            assert all(int(a[f]) == int(b[f]) for f in ("flag", "rid", "mrid", "pos", "mpos", "score", "n_cigar",
                                                         "seq_b", "seq_e")), (r, k)
            assert np.array_equal(a["cigar"][:nc], b["cigar"][:nc]), (r, k)


def _check_genome_records_oracle(d, og, q, nq, npair):
    from anchored_fusion_amd import discover, genome
    recs = d.q_recs[:nq * discover.MAX_REC * genome.REC_DTYPE.itemsize].cpu().numpy().view(genome.REC_DTYPE)
    recs = recs.reshape(nq, discover.MAX_REC)
    nrec = d.q_nh[:nq].cpu().numpy()
    lens = d.q_lens[:nq].cpu().numpy()
    r4, n4 = og.align_pe(q[:2 * npair], lens[:2 * npair], pe=oracle.default_pe(chunk_bases=d.chunk_bases, pair_base=0),
                         threads=16)
    r5, n5 = og.align_se(q[2 * npair:nq], lens[2 * npair:nq], id_base=0, threads=16)
    want_r, want_n = np.concatenate([r4, r5]), np.concatenate([n4, n5])
    assert np.array_equal(nrec, want_n), np.nonzero(nrec != want_n)[0][:10]
    assert (nrec >= 1).all() and 2 * npair > 100 and nq - 2 * npair > 100
    for r in range(nq):
        for k in range(min(int(nrec[r]), discover.MAX_REC)):
            a, b = recs[r, k], want_r[r, k]
            nc = int(a["n_cigar"])
            assert all(int(a[f]) == int(b[f]) for f in ("flag", "rid", "mrid", "pos", "mpos", "score", "n_cigar",
                                                         "seq_b", "seq_e")), (r, k)
            assert np.array_equal(a["cigar"][:nc], b["cigar"][:nc]), (r, k)


def _check_s5_s6(d, ref, reads, got, an, npair, nq):
    from anchored_fusion_amd import discover, genome
    from test_gpu_s5s6 import host_s5_s6
    n5 = nq - 2 * npair
    recs = d.q_recs[:nq * discover.MAX_REC * genome.REC_DTYPE.itemsize].cpu().numpy().view(genome.REC_DTYPE)
    recs = recs.reshape(nq, discover.MAX_REC)[2 * npair:]
    h = dict(got)
    h["cigar"] = h["cigar"].view(np.int32)
    fasta, split_sam, s6_fa = host_s5_s6(reads, h, an, recs, d.q_nh[2 * npair:nq].cpu().numpy(), ref.names)
    assert len(fasta) == n5
    n6 = int(d.s6["n"].item())
    assert n6 == len(s6_fa)
    rows, lens, src = d.s6["q"][:n6].cpu().numpy(), d.s6["lens"][:n6].cpu().numpy(), d.s6["src"][:n6].cpu().numpy()
    for k in range(n6):
        assert split_sam[k].split("\t")[0] == fasta[src[k]][0].split("$")[0]
        assert rows[k, :lens[k]].tobytes().decode() == s6_fa[k][1], k


def test_c3_full_size(anchor):
    """configs[2] at full size: 50 M pairs on the 3.09 Gbp world.  Properties: every read with an
    exact 19-mer of the anchor (either strand) passes the seed filter; the placed split-read
    tails' best hits lie in the embedded genes; the first two bwa chunks are bit-exact vs the
    oracle."""
    import torch

    from anchored_fusion_amd import discover
    from anchored_fusion_amd.shard import chunk_pairs
    W = _world(anchor, 1.0)
    ref = W.genome_index()
    tiles = W.tiles()
    # the 3.09 Gbp index by its defining properties on samples (tests/fm_checks.py): occurrence
    # totals, BWT blocks vs T[SA - 1], LF steps, suffix order over >= 4 kb
    from fm_checks import check_index
    summ_ix = check_index(ref.text, ref.sa, ref.occ, ref.l_pac, ref.primary(), seed=3, n_rows=1500, n_blocks=64)
    print("index checks", summ_ix)
    assert summ_ix["rows_above_2_31"] > 500 and summ_ix["undecided"] == 0
    _check_exact_reads_high(W, ref, L=150)
    N, L = 50_000_000, 150
    reads_t = W.simulate_pairs(N, read_len=L, seed=20251015)
    torch.cuda.synchronize()
    W.blob = None
    d = discover.CandidateDiscovery(anchor, ref, tiles, N, L, device=0)
    d.run(reads_t)
    summ = d.summary()
    assert summ["tmp1"] == summ["tmp2"] > 1000 and summ["anchored"] > 1_000_000
    assert summ["genome_cap_overflow"] == 0 and summ["queries_placed"] > 0.9 * summ["queries_s4_s5"]
    # oracle on the first two chunks (bwa's read ids and insert-size chunks are the same)
    m = 2 * chunk_pairs(L)
    sub = reads_t[:2 * m].cpu().numpy()
    got = {k: v[:2 * m].cpu().numpy() for k, v in d.out.items()}
    got["cigar"] = got["cigar"].view(np.uint32)
    assert_records_equal(got, oracle.OracleIndex(anchor).align_pairs(sub, threads=8), sub)
    # seed filter: no read holding an anchor 19-mer is dropped (sampled rows)
    comp = bytes.maketrans(b"ACGT", b"TGCA")
    an = anchor.upper()
    kmers = {an[i:i + 19] for i in range(len(an) - 18)}
    kmers |= {k[::-1].translate(comp) for k in kmers}
    rng = np.random.default_rng(1)
    rows = np.sort(rng.choice(2 * N, 40_000, replace=False))
    hits = d.out["hits"].cpu().numpy()[rows]
    sample = reads_t[torch.from_numpy(rows).cuda()].cpu().numpy()
    for r, h in zip(sample, hits):
        s = r.tobytes()
        if h == 0:
            assert not any(s[i:i + 19] in kmers for i in range(L - 18))
    # S6 (BLAT -minScore=20 of S5's survivors): best rows inside the anchor or a partner gene
    # locus (exons and introns)
    spans = [(W.names.index(v[0][0]), v[0][1] - 1000, v[-1][2] + 1000) for v in W.loci.values()]
    _, nh, best = d.s6_best_hits()
    placed = np.nonzero(nh > 0)[0]
    inside = 0
    for t in placed:
        loc = tiles.locate(best[t]["t_start"], best[t]["t_end"])
        inside += loc is not None and any(k == loc[0] and s <= loc[1] < e for k, s, e in spans)
    print(f"S6 queries placed {len(placed)}, best hit in a gene locus {inside}")
    assert len(placed) > 10_000 and inside >= 0.95 * len(placed)
    d.close()
    ref.close()
    tiles.close()


def _check_exact_reads_high(W, ref, L, n=3000):
    """Error-free reads cut from the genome beyond 2^31 (forward pac coordinates; their reverse
    complements too): every one maps with CIGAR L M and score L (S5's call), at a locus whose bases
    equal the read (a repeat may place it elsewhere with the same score), and most at their origin."""
    import torch
    comp = bytes.maketrans(b"ACGT", b"TGCA")
    rng = np.random.default_rng(11)
    offs = np.asarray(W.offsets, np.int64)
    lens = np.asarray(W.lens, np.int64)
    reads, origin = [], []
    while len(reads) < n:
        g = int(rng.integers(1 << 31, int(offs[-1] + lens[-1]) - L))
        k = int(np.searchsorted(offs, g, side="right") - 1)
        if g + L > offs[k] + lens[k]:
            continue
        s = W.blob[g:g + L].cpu().numpy().tobytes()
        if b"N" in s:
            continue
        rev = len(reads) % 2 == 1
        reads.append(s[::-1].translate(comp) if rev else s)
        origin.append((k, g - int(offs[k]), rev))
    arr = np.frombuffer(b"".join(reads), np.uint8).reshape(n, L)
    recs, nrec = ref.align_se(arr, np.full(n, L, np.int32))
    at_origin = 0
    for i in range(n):
        r = recs[i, 0]
        assert (int(r["flag"]) & 4) == 0 and int(r["score"]) == L and int(r["n_cigar"]) == 1, i
        assert int(r["cigar"][0]) == (L << 4), i
        k, p = int(r["rid"]), int(r["pos"])
        g0 = int(offs[k]) + p
        locus = W.blob[g0:g0 + L].cpu().numpy().tobytes()
        rev = bool(int(r["flag"]) & 0x10)
        assert (locus[::-1].translate(comp) if rev else locus) == reads[i], i
        at_origin += (k, p, rev) == origin[i]
    print(f"exact reads beyond 2^31: {n} mapped, {at_origin} at their origin")
    assert at_origin > 0.8 * n
    torch.cuda.synchronize()


def test_discovery_rank_shard_and_search(anchor, monkeypatch):
    """A rank's shard (pair_base on the bwa chunk grid, as bench.py's ranks run it): records
    bit-exact vs the oracle with the same read ids; then the product's multi-GPU step
    (dist_discover.search) over a one-rank RCCL group (AF_DIST_COLLECTIVES=1: every all-gather /
    all-to-all through RCCL on device tensors) gives the single-process pass's counts, S4 records
    and survivors, with global read rows."""
    import os
    import socket

    import torch
    import torch.distributed as dist

    from anchored_fusion_amd import discover, dist_discover
    from anchored_fusion_amd.genome import MAX_REC, REC_DTYPE
    from anchored_fusion_amd.shard import chunk_pairs
    W = _world(anchor, 0.02)
    ref = W.genome_index()
    tiles = W.tiles()
    n, pb = 60_000, 3 * chunk_pairs(150)
    reads_t = W.simulate_pairs(n, read_len=150, seed=13, pair_base=pb)
    d = discover.CandidateDiscovery(anchor, ref, tiles, n, 150, device=0, inflight=2, batch_chunks=1, pair_base=pb)
    d.run(reads_t)
    torch.cuda.synchronize()
    reads = reads_t.cpu().numpy()
    got = {k: v.cpu().numpy() for k, v in d.out.items()}
    got["cigar"] = got["cigar"].view(np.uint32)
    assert_records_equal(got, oracle.OracleIndex(anchor).align_pairs(reads, threads=8, pair_base=pb), reads)
    q = d.q[:int(d.n_q.item())].cpu().numpy()
    _check_genome_records(d, ref, q, q.shape[0], d.counts["s4_pairs"])
    # the single-process pass's products
    counts1 = dict(d.counts)
    npair = counts1["s4_pairs"]
    words = REC_DTYPE.itemsize // 4
    recs1 = d.q_recs.view(torch.int32)[:2 * npair * MAX_REC * words].reshape(2 * npair, MAX_REC, words).clone()
    nrec1 = d.q_nh[:2 * npair].clone()
    n6 = int(d.s6["n"].item())
    surv_rows1 = (d.q_rows[2 * npair:][d.s6["src"][:n6].long()].long() + 2 * pb).cpu()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(port))
    monkeypatch.setenv("AF_DIST_COLLECTIVES", "1")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        res, counts = dist_discover.search(d.attach(reads_t), pb, 0, 1, device="cuda:0")
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    for k in ("tmp1", "tmp2", "s5_split_reads", "s4_pairs"):
        assert counts[k] == counts1[k], k
    assert counts["s6_queries"] == n6 > 0
    _, _, recs, nrec, _ = res["s4"]
    assert torch.equal(nrec.cpu(), nrec1.cpu().to(nrec.dtype))
    live = torch.arange(MAX_REC)[None, :] < nrec1.cpu().clamp(max=MAX_REC).long()[:, None]
    assert torch.equal(recs.cpu()[live], recs1.cpu()[live])
    # the survivors in ordinal order with their global read rows (the last two words of a row)
    grow = dist_discover._i64(res["surv"][:, -2:]).cpu()
    assert torch.equal(torch.sort(grow).values, torch.sort(surv_rows1).values)
    assert (grow >= 2 * pb).all() and (grow < 2 * (pb + n)).all()
    d.close()
    ref.close()
    tiles.close()
