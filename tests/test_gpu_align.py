"""GPU parity tests: the HIP path (libafgpu.so via the C-ABI) against the CPU oracle.

Bar: bit-exact on every per-read field (flag, pos, score, n_cigar, CIGAR ops, seed-filter
hits) -- this is integer/index work.  Sizes are chosen so the oracle finishes in seconds;
the full-size config is checked through size-independent properties.
"""
import numpy as np
import pytest

import oracle
from cases import edge_pairs, ragged, synthetic_pairs
from helpers import assert_records_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def aligner(anchor):
    from anchored_fusion_amd.align import AnchorAligner
    a = AnchorAligner(anchor, device=0)
    yield a
    a.close()


@pytest.fixture(scope="module")
def oidx(anchor):
    return oracle.OracleIndex(anchor)


def _both(aligner, oidx, reads, lens=None, pair_base=0):
    g = aligner.align_pairs(reads, lens, pair_base=pair_base).as_dict()
    r = oidx.align_pairs(reads, lens, threads=8, pair_base=pair_base, chunk_bases=int(aligner.pe.chunk_bases))
    return g, r


def test_filter_table_matches_oracle(aligner, oidx):
    assert np.array_equal(aligner.filter_table(), oidx.filter_table())


def test_bundled_parity(aligner, oidx, bundled_pairs):
    names, reads, lens = bundled_pairs
    g, r = _both(aligner, oidx, reads, lens)
    assert_records_equal(g, r, reads)
    assert ((g["flag"] & 4) == 0).sum() == 1264  # 1,261 seeded + 3 rescued mates (test_oracle.py)


def test_align_fastq_streamed_matches_oracle(aligner, oidx, bundled_pairs):
    # native FASTQ.gz ingest overlapped with alignment, in 3,000-pair batches (the last ragged)
    import os
    gold = os.path.join(os.path.dirname(__file__), "golden")
    names, reads, lens, res = aligner.align_fastq(os.path.join(gold, "test_sample_1.fastq.gz"),
                                                  os.path.join(gold, "test_sample_2.fastq.gz"), batch_pairs=3000)
    n0, r0, l0 = bundled_pairs
    assert lens is None and l0 is None and (reads == r0).all() and list(names) == list(n0)
    assert_records_equal(res.as_dict(), oidx.align_pairs(reads, None, threads=8), reads)


def test_rescue_parity(aligner, oidx, anchor):
    """mem_matesw on the GPU: the unseedable mate is rescued exactly as by the oracle."""
    from cases import rescue_pairs
    reads, probe = rescue_pairs(anchor)
    g, r = _both(aligner, oidx, reads)
    assert_records_equal(g, r, reads)
    assert g["hits"][2 * probe + 1] == 0 and not g["flag"][2 * probe + 1] & 4


def test_tie_break_parity(anchor):
    """Equal-score hits on a duplicated segment: the hash_64(read id) primary choice, for several
    pair_base values (bwa's global read ids)."""
    from anchored_fusion_amd.align import AnchorAligner
    from cases import repeat_anchor_pairs
    anc2, reads = repeat_anchor_pairs(anchor)
    ix = oracle.OracleIndex(anc2)
    picks = set()
    with AnchorAligner(anc2, device=0) as a:
        for base in (0, 1, 7, 1000, 123456, (1 << 31) - 5):
            g, r = _both(a, ix, reads, pair_base=base)
            assert_records_equal(g, r, reads)
            picks.add(tuple(g["pos"][0::2]))
    assert len(picks) > 1


@pytest.mark.parametrize("chunk_pairs", [6, 250, 1013])
def test_chunked_insert_stats_parity(anchor, oidx, chunk_pairs):
    """Several bwa chunks in one batch (insert-size statistics per chunk), uniform and ragged."""
    from anchored_fusion_amd import _lib
    from anchored_fusion_amd.align import AnchorAligner
    reads, _, _ = synthetic_pairs(anchor, 3000, 100, seed=61, fusion_frac=0.9)
    with AnchorAligner(anchor, device=0, pe=_lib.default_pe(chunk_bases=200 * chunk_pairs)) as a:
        g, r = _both(a, oidx, reads)
        assert_records_equal(g, r, reads)
        rr, lens = ragged(reads, 62)
        g, r = _both(a, oidx, rr, lens)
        assert_records_equal(g, r, rr)


def test_tandem_repeat_parity(aligner, oidx, anchor):
    """Reads of a tandem repeat that occurs in the anchor: many equal-scoring regions."""
    from cases import tandem_pairs
    reads = tandem_pairs(anchor)
    g, r = _both(aligner, oidx, reads)
    assert_records_equal(g, r, reads)


def test_edge_parity(aligner, oidx, anchor):
    reads, lens = edge_pairs(anchor)
    g, r = _both(aligner, oidx, reads, lens)
    assert_records_equal(g, r, reads)


@pytest.mark.parametrize("read_len,seed", [(100, 1), (101, 2), (150, 3), (76, 4), (250, 5)])
def test_synthetic_parity(aligner, oidx, anchor, read_len, seed):
    reads, _, _ = synthetic_pairs(anchor, 4000, read_len, seed=seed)
    g, r = _both(aligner, oidx, reads)
    assert_records_equal(g, r, reads)
    assert ((g["flag"] & 4) == 0).sum() > 1000


def test_high_error_parity(aligner, oidx, anchor):
    """Many mismatches and indels: exercises band inference, global DP and traceback."""
    reads, _, _ = synthetic_pairs(anchor, 3000, 150, seed=9, err=0.06, indel_frac=0.3)
    g, r = _both(aligner, oidx, reads)
    assert_records_equal(g, r, reads)


def test_ragged_parity(aligner, oidx, anchor):
    reads, _, _ = synthetic_pairs(anchor, 3000, 150, seed=21)
    rr, lens = ragged(reads, 22)
    g, r = _both(aligner, oidx, rr, lens)
    assert_records_equal(g, r, rr)


def test_empty_and_tiny_batches(aligner, oidx, anchor):
    reads, lens = edge_pairs(anchor)
    g, r = _both(aligner, oidx, reads[:2], lens[:2])
    assert_records_equal(g, r)
    e = aligner.align_pairs(np.zeros((0, 100), dtype=np.uint8))
    assert len(e) == 0


def test_device_api_matches_host_api(aligner, anchor):
    import torch
    reads, _, _ = synthetic_pairs(anchor, 5000, 100, seed=31)
    host = aligner.align_pairs(reads).as_dict()
    dev = torch.device("cuda:0")
    nr = reads.shape[0]
    rt = torch.from_numpy(reads).to(dev)
    out = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
    out["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    aligner.align_pairs_device(rt, nr // 2, reads.shape[1], out, stream=s)
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in out.items()}
    got["cigar"] = got["cigar"].view(np.uint32)
    assert_records_equal(got, host, reads)


def test_aligner_group_matches_oracle(anchor, oidx):
    """AlignerGroup (the bench's schedule): three different batches in flight, two groups in a
    row over reused buffers, every batch's records equal to the oracle's; ragged lengths too."""
    import torch
    from anchored_fusion_amd.align import AlignerGroup
    dev = torch.device("cuda:0")
    cases = [synthetic_pairs(anchor, 3000, 100, seed=41 + k)[0] for k in range(3)]
    rg, rl = ragged(*synthetic_pairs(anchor, 2000, 150, seed=44)[:1], seed=45)
    grp = AlignerGroup(anchor, device=0, inflight=3)
    try:
        def outs(nr):
            o = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
            o["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
            return o
        done = None
        for group in ([(c, None) for c in cases], [(cases[2], None), (rg, rl)]):
            bufs = [outs(r.shape[0]) for r, _ in group]
            batch = []
            for (r, ln), o in zip(group, bufs):
                b = (torch.from_numpy(r).to(dev), r.shape[0] // 2, r.shape[1], o)
                batch.append(b if ln is None else b + (torch.from_numpy(ln).to(dev),))
            done = grp.run_device(batch, wait=done)
            grp.join(done)
            torch.cuda.synchronize()
            for (r, ln), o in zip(group, bufs):
                got = {k: v.cpu().numpy() for k, v in o.items()}
                got["cigar"] = got["cigar"].view(np.uint32)
                assert_records_equal(got, oidx.align_pairs(r, ln, threads=8), r)
    finally:
        grp.close()


def test_full_size_properties(aligner, anchor):
    """Config-2 size (1 M pairs x 2x100): properties that do not need the oracle."""
    import torch
    from anchored_fusion_amd import simulate as sim
    _, reads, truth, world = sim.fusion_reads(anchor, 1_000_000, read_len=100, fusion_frac=0.05, seed=20251015)
    dev = torch.device("cuda:0")
    nr = reads.shape[0]
    rt = torch.from_numpy(reads).to(dev)
    out = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
    out["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
    aligner.align_pairs_device(rt, nr // 2, 100, out)
    torch.cuda.synchronize()
    f = out["flag"].cpu().numpy()
    h = out["hits"].cpu().numpy()
    mapped = (f & 4) == 0
    # the filter never drops a seeded read: a mapped read without a K1 hit is a rescued mate
    rescued = mapped & (h == 0)
    assert (~np.repeat(((f[0::2] | f[1::2]) & 4) != 0, 2) | ~rescued).all()
    assert rescued.sum() < 0.01 * mapped.sum()
    # bwa's chunks (50,000 pairs of 2x100) are independent: two of them against the oracle alone
    got = {k: v.cpu().numpy() for k, v in out.items()}
    got["cigar"] = got["cigar"].view(np.uint32)
    for c in (0, 10):
        lo, hi = 50_000 * c, 50_000 * (c + 1)
        want = oracle.OracleIndex(anchor).align_pairs(reads[2 * lo:2 * hi], threads=16, pair_base=lo)
        assert_records_equal({k: v[2 * lo:2 * hi] for k, v in got.items()}, want, reads[2 * lo:2 * hi])
    nf = len(world["fusions"])
    from_fusion = np.repeat(truth["tid"] < nf, 2)
    assert mapped[~from_fusion].mean() < 1e-3          # background essentially never maps
    assert mapped[from_fusion].mean() > 0.3            # anchor-side reads of fusions do
    # idempotence: a second run gives identical records
    f2 = out["flag"].clone()
    aligner.align_pairs_device(rt, nr // 2, 100, out)
    torch.cuda.synchronize()
    assert torch.equal(f2, out["flag"])


@pytest.mark.parametrize("stride", [16, 17, 20, 27, 28, 29, 33, 64, 99, 100, 101, 150, 251, 320])
def test_seed_filter_strides(aligner, oidx, anchor, stride):
    """K1 alone: per-read Bloom hits equal the oracle's for every stride class (reads that end
    inside a 16-byte chunk, chunks spanning two reads, strides below 28 where one chunk's
    k-mers can straddle a read end), on a batch that leaves a partial last tile."""
    import torch
    from anchored_fusion_amd import simulate as sim
    n = 2 * 2048 * 3 + 777
    L = min(stride, 150)
    reads = np.full((n, stride), ord("N"), dtype=np.uint8)
    r, _, _ = synthetic_pairs(anchor, n // 2 + 1, max(L, 40), seed=stride)
    reads[:, :min(L, stride)] = r[:n, :min(L, stride)]
    rng = np.random.default_rng(stride)
    noise = rng.random(reads.shape) < 0.3                    # background-like bytes too
    reads[noise] = np.frombuffer(sim.random_seq(rng, int(noise.sum())), dtype=np.uint8)
    dev = torch.device("cuda:0")
    rt = torch.from_numpy(reads).to(dev)
    hits = torch.zeros(n, dtype=torch.int32, device=dev)
    aligner.seed_filter_device(rt, n, stride, hits)
    torch.cuda.synchronize()
    want = oidx.seed_filter(reads)
    got = hits.cpu().numpy()
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert aligner.last_candidates() == int((want > 0).sum())


@pytest.mark.parametrize("stride", [20, 33, 100, 151, 320])
def test_seed_filter_ragged_strides(aligner, oidx, anchor, stride):
    """K1's ragged path (per-read lengths, k_seed_ragged): hits equal the oracle's for reads of
    every length 0..stride, including lengths below one 16-mer."""
    import torch
    n = 2 * 2048 * 2 + 313
    reads = np.full((n, stride), ord("N"), dtype=np.uint8)
    r, _, _ = synthetic_pairs(anchor, n // 2 + 1, min(max(stride, 40), 250), seed=1000 + stride)
    w = min(stride, r.shape[1])
    reads[:, :w] = r[:n, :w]
    rng = np.random.default_rng(stride)
    lens = rng.integers(0, stride + 1, size=n).astype(np.int32)
    lens[:64] = np.arange(64) % (stride + 1)
    dev = torch.device("cuda:0")
    rt = torch.from_numpy(reads).to(dev)
    lt = torch.from_numpy(lens).to(dev)
    hits = torch.zeros(n, dtype=torch.int32, device=dev)
    aligner.seed_filter_device(rt, n, stride, hits, lens_t=lt)
    torch.cuda.synchronize()
    want = oidx.seed_filter(reads, lens)
    got = hits.cpu().numpy()
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert aligner.last_candidates() == int((want > 0).sum())


def _random_records(n, seed, max_pos=300):
    """Flag/pos columns with bwa's pair conventions (as test_consumers.test_partition_matches_full_sort)."""
    rng = np.random.default_rng(seed)
    flag = np.zeros(n, np.int32)
    pos = np.full(n, -1, np.int32)
    m = rng.random((n // 2, 2)) < 0.3
    rv = rng.random((n // 2, 2)) < 0.5
    x = rng.integers(0, max_pos, (n // 2, 2))
    sec = rng.random((n // 2, 2)) < 0.02
    for k in (0, 1):
        f = np.full(n // 2, 0x1 | (0x40 if k == 0 else 0x80), np.int32)
        f |= np.where(m[:, k], np.where(rv[:, k], 0x10, 0), 0x4).astype(np.int32)
        f |= np.where(~m[:, 1 - k], 0x8, np.where(rv[:, 1 - k], 0x20, 0)).astype(np.int32)
        f |= np.where(sec[:, k] & m[:, k], 0x100, 0).astype(np.int32)
        flag[k::2] = f
        pos[k::2] = np.where(m[:, k], x[:, k], np.where(m[:, 1 - k], x[:, 1 - k], -1))
    return flag, pos


@pytest.mark.parametrize("n,seed,max_pos", [(2, 1, 5), (20000, 5, 300), (400000, 6, 7000), (1 << 20, 7, 40)])
def test_partition_device_matches_host(aligner, n, seed, max_pos):
    """S3 on the device (af_partition_device) vs align.partition: identical row lists."""
    import torch
    from anchored_fusion_amd.align import AlignResult, partition
    flag, pos = _random_records(n, seed, max_pos)
    z = np.zeros(n, np.int32)
    want = partition(AlignResult(flag, pos, z, z, np.zeros((n, 1), np.uint32), z))
    dev = torch.device("cuda:0")
    t1, t2, an, cnt = aligner.partition_device(torch.from_numpy(flag).to(dev), torch.from_numpy(pos).to(dev))
    c = cnt.cpu().numpy()
    for g, k, w in zip((t1, t2, an), c, want):
        assert np.array_equal(g[:k].cpu().numpy(), w)


def test_partition_device_on_s2_records(aligner, anchor):
    """S3 after S2 on the device, both in HBM: equal to the host partition of the same records."""
    import torch
    from anchored_fusion_amd.align import AlignResult, partition
    reads, _, _ = synthetic_pairs(anchor, 20000, 150, seed=71, fusion_frac=0.5)
    dev = torch.device("cuda:0")
    nr = reads.shape[0]
    out = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
    out["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
    aligner.align_pairs_device(torch.from_numpy(reads).to(dev), nr // 2, 150, out)
    t1, t2, an, cnt = aligner.partition_device(out["flag"], out["pos"])
    got = {k: v.cpu().numpy() for k, v in out.items()}
    want = partition(AlignResult(got["flag"], got["pos"], got["score"], got["n_cigar"], got["cigar"], got["hits"]))
    c = cnt.cpu().numpy()
    assert c[2] > 1000
    for g, k, w in zip((t1, t2, an), c, want):
        assert np.array_equal(g[:k].cpu().numpy(), w)


@pytest.mark.parametrize("windows", ["1", "3"])
def test_k3c_rescue_jobs_parity(anchor, oidx, monkeypatch, windows):
    """K3c's heavy pairs (at least AF_S2_SPEC_WINDOWS mate-rescue windows, read when the context
    is made): their rescue SWs computed ahead as grid-wide jobs (k_s2_pe_jobs), the pair's walk
    taking the results (k_s2_pairs mode 2) -- every record equal to the oracle's, on the rescue,
    tandem-repeat and fusion-rich cases."""
    from anchored_fusion_amd.align import AnchorAligner
    from cases import rescue_pairs, tandem_pairs
    monkeypatch.setenv("AF_S2_SPEC_WINDOWS", windows)
    sets = [rescue_pairs(anchor)[0], tandem_pairs(anchor), synthetic_pairs(anchor, 3000, 150, seed=71, fusion_frac=0.9)[0]]
    with AnchorAligner(anchor, device=0) as a:
        for reads in sets:
            g, r = _both(a, oidx, reads)
            assert_records_equal(g, r, reads)
