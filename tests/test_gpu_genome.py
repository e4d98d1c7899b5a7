"""The genome calls S4 / S5 on the GPU (csrc/fmindex.hip, csrc/bwa_genome.hip) against the CPU
restatement (oracle/bwa_pe.c, FM mode) -- bit-exact.

* the index: bns_fasta2bntseq's text (lrand48 for ambiguous bases) and the suffix array, equal
  row for row on a repeat-rich genome (young Alu-like subfamily above max_occ, a satellite array,
  an exact 3 kb duplication, N runs);
* S5 (`bwa mem -M genome reads.fa`, functions.py:716): regions after mem_align1_core and every
  SAM record (flags, contigs, positions, CIGARs with -M hard clips, SEQ slices) on chimeric and
  plain reads with errors, indels and N;
* S4 (`bwa mem -M genome fq1 fq2`, AF:188): every record of every pair, with the per-chunk
  insert-size statistics, mate rescue and pairing.
"""
import numpy as np
import pytest

import afpkg  # noqa: F401
import oracle
from genome_world import make_genome, sample_pairs, sample_reads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world():
    contigs = make_genome()
    from anchored_fusion_amd.genome import GenomeIndex
    return contigs, oracle.OracleGenome(contigs), GenomeIndex(contigs, device=0)


def test_index_equals_oracle(world):
    _, og, gg = world
    assert gg.l_pac == og.l_pac
    assert np.array_equal(gg.text(), og.text())
    assert gg.primary() == og.primary()
    sa_o, sa_g = og.sa(), gg.sa()
    bad = np.nonzero(sa_o != sa_g)[0]
    assert bad.size == 0, f"{bad.size} suffix-array rows differ, first {bad[:5]}"


def _rec_equal(a, b, n):
    for k in range(n):
        x, y = a[k], b[k]
        for f in ("flag", "rid", "mrid", "pos", "mpos", "score", "n_cigar", "seq_b", "seq_e"):
            if int(x[f]) != int(y[f]):
                return f"record {k} field {f}: {int(x[f])} != {int(y[f])}"
        nc = int(x["n_cigar"])
        if not np.array_equal(x["cigar"][:nc], y["cigar"][:nc]):
            return f"record {k} cigar"
    return None


def _iv_sets_equal(io, no, ig, ng):
    """Per read: the same count and the same intervals (sorted by qb, qe, SA row, size: equal
    (qb, qe) keys hold identical intervals, in any order)."""
    assert np.array_equal(no, ng), np.nonzero(no != ng)[0][:10]
    for r in range(len(no)):
        k = min(int(no[r]), io.shape[1])
        a, b = io[r, :k], ig[r, :k]
        a = a[np.lexsort((a[:, 1], a[:, 0], a[:, 3], a[:, 2]))]
        b = b[np.lexsort((b[:, 1], b[:, 0], b[:, 3], b[:, 2]))]
        assert np.array_equal(a, b), (r, a[:4], b[:4])


def test_intervals_equal_oracle(world):
    """G1 (mem_collect_intv: SMEMs, re-seeding, bwt_seed_strategy1) interval by interval."""
    contigs, og, gg = world
    reads, lens = sample_reads(contigs, 800, seed=20, chimeric=0.4)
    io, no = og.intervals(reads, lens, threads=8)
    ig, ng = gg.intervals(reads, lens)
    _iv_sets_equal(io, no, ig, ng)
    assert no.mean() > 4


def test_se_regions_equal_oracle(world):
    contigs, og, gg = world
    reads, lens = sample_reads(contigs, 400, seed=21)
    ro, no = og.regions(reads, lens, max_reg=64, threads=8)
    rg, ng = gg.regions(reads, lens, max_reg=64)
    assert np.array_equal(no, ng), np.nonzero(no != ng)[0][:10]
    for r in range(len(no)):
        for k in range(min(no[r], 64)):
            o = ro[r, k]
            g = rg[r, k]
            want = (o["rb"], o["re"], o["qb"], o["qe"], o["rid"], o["score"], o["truesc"], o["w"], o["seedcov"],
                    o["seedlen0"])
            assert tuple(int(v) for v in want) == tuple(int(v) for v in g[:10]), (r, k)


@pytest.mark.parametrize("arr", ["0", "3"])
def test_chain_modes_equal_oracle(world, monkeypatch, arr):
    """mem_chain's two modes (bwa_genome.hip g_mem_chain): the sorted chain array in LDS (default)
    and the kbtree, which a read restarts on at a second chain with an existing pos or past the
    array's limit -- forced here for every read (AF_G_CHAIN_ARR=0, which also runs mem_chain_flt's
    chunk scan instead of its grouped scan) or past 3 chains (most multi-chain reads restart).
    Regions and records equal the oracle's either way."""
    monkeypatch.setenv("AF_G_CHAIN_ARR", arr)
    contigs, og, gg = world
    reads, lens = sample_reads(contigs, 400, seed=31, chimeric=0.4)
    ro, no = og.regions(reads, lens, max_reg=64, threads=8)
    rg, ng = gg.regions(reads, lens, max_reg=64)
    assert np.array_equal(no, ng), np.nonzero(no != ng)[0][:10]
    for r in range(len(no)):
        for k in range(min(no[r], 64)):
            o = ro[r, k]
            want = (o["rb"], o["re"], o["qb"], o["qe"], o["rid"], o["score"], o["truesc"], o["w"], o["seedcov"],
                    o["seedlen0"])
            assert tuple(int(v) for v in want) == tuple(int(v) for v in rg[r, k][:10]), (r, k)
    so, sn = og.align_se(reads, lens, id_base=7, threads=8)
    sg, sgn = gg.align_se(reads, lens, id_base=7)
    assert np.array_equal(sn, sgn)
    for r in range(len(sn)):
        msg = _rec_equal(so[r], sg[r], min(sn[r], 8))
        assert msg is None, (r, msg)


def test_wave_introsort_equals_klib():
    """bwa_dev.h wave_introsort (mem_chain_flt's sort of (weight << 32 | index) keys by weight,
    descending: ties everywhere) returns klib's introsort's exact order, through the test hook
    af_debug_wave_introsort; lists of 3..2,048 keys with 1..1,000 distinct weights."""
    import ctypes
    from anchored_fusion_amd import _lib
    L = _lib.lib()
    L.af_debug_wave_introsort.restype = ctypes.c_int
    L.af_debug_wave_introsort.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
    rng = np.random.default_rng(41)
    for n in (3, 17, 64, 65, 100, 257, 600, 1024, 1106, 2048):
        for nw in (1, 2, 5, 40, 1000):
            w = rng.integers(0, nw, n).astype(np.uint64)
            keys = (w << np.uint64(32)) | np.arange(n, dtype=np.uint64)
            a = np.zeros(n, np.uint64)
            b = np.zeros(n, np.uint64)
            assert L.af_debug_wave_introsort(keys.ctypes.data, n, a.ctypes.data, b.ctypes.data) == 0
            assert np.array_equal(a, b), (n, nw, np.nonzero(a != b)[0][:5])
            assert np.all(np.diff((a >> np.uint64(32)).astype(np.int64)) <= 0)


def test_se_records_equal_oracle(world):
    contigs, og, gg = world
    reads, lens = sample_reads(contigs, 600, seed=22, chimeric=0.4)
    ro, no = og.align_se(reads, lens, id_base=7, threads=8)
    rg, ng = gg.align_se(reads, lens, id_base=7)
    assert np.array_equal(no, ng)
    for r in range(len(no)):
        msg = _rec_equal(ro[r], rg[r], min(no[r], 8))
        assert msg is None, (r, msg)
    assert gg.stats()["cap_overflow"] == 0
    n_supp = int(((rg["flag"] & 0x100) != 0).sum())
    assert n_supp > 20 and int(((rg[:, 0]["flag"] & 4) == 0).sum()) > 500


def test_pe_records_equal_oracle(world):
    contigs, og, gg = world
    reads = sample_pairs(contigs, 1500, seed=23)
    lens = np.full(reads.shape[0], reads.shape[1], np.int32)
    # two bwa chunks (insert-size statistics per chunk) at 300 kbase
    pe_o = oracle.default_pe(chunk_bases=300_000, pair_base=4)
    ro, no = og.align_pe(reads, lens, pe=pe_o, threads=8)
    from anchored_fusion_amd import _lib
    rg, ng = gg.align_pe(reads, lens, pe=_lib.default_pe(chunk_bases=300_000, pair_base=4))
    assert np.array_equal(no, ng)
    for r in range(len(no)):
        msg = _rec_equal(ro[r], rg[r], min(no[r], 8))
        assert msg is None, (r, msg)
    assert int(((rg[:, 0]["flag"] & 2) != 0).sum()) > 1500  # proper pairs found


def test_pe_rescue_case_equals_oracle():
    """tests/test_genome_rescue_blocks.py's crafted pairs (a mate placeable only by mem_matesw,
    2.5 kb inserts): the kernel's records equal the oracle's with rescue on and off."""
    from anchored_fusion_amd import _lib
    from anchored_fusion_amd.genome import GenomeIndex
    from test_genome_rescue_blocks import L, crafted
    contigs, reads, _ = crafted()
    og, gg = oracle.OracleGenome(contigs), GenomeIndex(contigs, device=0)
    try:
        lens = np.full(reads.shape[0], L, np.int32)
        for matesw in (50, 0):
            pe_o = oracle.default_pe()
            pe_o.max_matesw = matesw
            pe_g = _lib.default_pe()
            pe_g.max_matesw = matesw
            ro, no = og.align_pe(reads, lens, pe=pe_o, pair_base=0, threads=8)
            rg, ng = gg.align_pe(reads, lens, pe=pe_g)
            assert np.array_equal(no, ng), matesw
            for r in range(len(no)):
                msg = _rec_equal(ro[r], rg[r], min(no[r], 8))
                assert msg is None, (matesw, r, msg)
            probe = rg[len(reads) - 1, 0]
            assert bool(probe["flag"] & 4) == (matesw == 0)
    finally:
        gg.close()


def test_pe_se_one_launch_equals_oracle(world):
    """af_genome_align_pe_se_device: S4's pairs and S5's queries through one launch of the seed /
    region kernels, S4's records on a second stream -- every record equal to the oracle's two
    separate calls (S4 with its chunk grid, S5 with its read ids)."""
    import torch

    from anchored_fusion_amd import _lib
    from anchored_fusion_amd.genome import MAX_REC, REC_DTYPE
    contigs, og, gg = world
    pairs = sample_pairs(contigs, 700, seed=31)
    se, se_lens = sample_reads(contigs, 500, seed=32, chimeric=0.4)
    L = max(pairs.shape[1], se.shape[1])
    reads = np.zeros((pairs.shape[0] + se.shape[0], L), np.uint8)
    reads[:pairs.shape[0], :pairs.shape[1]] = pairs
    reads[pairs.shape[0]:, :se.shape[1]] = se
    lens = np.concatenate([np.full(pairs.shape[0], pairs.shape[1], np.int32), se_lens.astype(np.int32)])
    pe_o = oracle.default_pe(chunk_bases=150_000, pair_base=2)
    ro4, no4 = og.align_pe(reads[:pairs.shape[0], :pairs.shape[1]], lens[:pairs.shape[0]], pe=pe_o, threads=8)
    ro5, no5 = og.align_se(se, se_lens, id_base=11, threads=8)
    dev = torch.device("cuda:0")
    n = reads.shape[0]
    rt = torch.from_numpy(reads).to(dev)
    lt = torch.from_numpy(lens).to(dev)
    recs = torch.zeros(n * MAX_REC * REC_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    nrec = torch.zeros(n, dtype=torch.int32, device=dev)
    s_a, s_b = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    s_a.wait_stream(torch.cuda.current_stream(dev))  # the zeroed recs / nrec and the uploads come first
    gg.align_pe_se_device(rt, pairs.shape[0] // 2, se.shape[0], L, lt, recs, nrec,
                          pe_s4=_lib.default_pe(chunk_bases=150_000, pair_base=2), pe_s5=_lib.default_pe(),
                          se_id_base=11, stream=s_a, stream_pe=s_b)
    torch.cuda.synchronize(dev)
    rg = recs.cpu().numpy().view(REC_DTYPE).reshape(n, MAX_REC)
    ng = nrec.cpu().numpy()
    P = pairs.shape[0]
    assert np.array_equal(ng[:P], no4) and np.array_equal(ng[P:], no5)
    for r in range(P):
        msg = _rec_equal(ro4[r], rg[r], min(no4[r], 8))
        assert msg is None, ("S4", r, msg)
    for r in range(se.shape[0]):
        msg = _rec_equal(ro5[r], rg[P + r], min(no5[r], 8))
        assert msg is None, ("S5", r, msg)


def test_heavy_path_equals_oracle(world, monkeypatch):
    """G2's heavy-read path (kept chains extended one job per chain, k_g_ext_jobs, then bwa's walk
    over the jobs' regions, k_g_heavy) forced for every read (AF_G_HEAVY_CHAINS=1, read when the
    context is made): regions, S5 records and S4 records equal the oracle's."""
    from anchored_fusion_amd import _lib
    from anchored_fusion_amd.genome import GenomeIndex
    contigs, og, _ = world
    monkeypatch.setenv("AF_G_HEAVY_CHAINS", "1")
    gh = GenomeIndex(contigs, device=0)
    try:
        reads, lens = sample_reads(contigs, 500, seed=41, chimeric=0.4)
        ro, no = og.regions(reads, lens, max_reg=64, threads=8)
        rg, ng = gh.regions(reads, lens, max_reg=64)
        assert np.array_equal(no, ng), np.nonzero(no != ng)[0][:10]
        for r in range(len(no)):
            for k in range(min(no[r], 64)):
                o = ro[r, k]
                want = (o["rb"], o["re"], o["qb"], o["qe"], o["rid"], o["score"], o["truesc"], o["w"], o["seedcov"],
                        o["seedlen0"])
                assert tuple(int(v) for v in want) == tuple(int(v) for v in rg[r, k][:10]), (r, k)
        so, sno = og.align_se(reads, lens, id_base=3, threads=8)
        sg, sng = gh.align_se(reads, lens, id_base=3)
        assert np.array_equal(sno, sng)
        for r in range(len(sno)):
            msg = _rec_equal(so[r], sg[r], min(sno[r], 8))
            assert msg is None, (r, msg)
        pairs = sample_pairs(contigs, 600, seed=42)
        plens = np.full(pairs.shape[0], pairs.shape[1], np.int32)
        po, pno = og.align_pe(pairs, plens, pe=oracle.default_pe(chunk_bases=200_000, pair_base=1), threads=8)
        pg, png = gh.align_pe(pairs, plens, pe=_lib.default_pe(chunk_bases=200_000, pair_base=1))
        assert np.array_equal(pno, png)
        for r in range(len(pno)):
            msg = _rec_equal(po[r], pg[r], min(pno[r], 8))
            assert msg is None, (r, msg)
    finally:
        gh.close()


@pytest.mark.parametrize("max_ext", [0, 1, 300])
def test_g1_wave_path_equals_oracle(world, monkeypatch, max_ext):
    """G1's heavy reads (k_g_seeds_wave: one wave per read, a position's backward-scan entries
    extended at once) -- every read handed off after its first FM extension (max_ext 1; the
    default for calls of few reads per CU), the reads past 300 extensions, or none (0: the lane
    path alone): intervals, S5 records and S4 records equal the oracle's."""
    from anchored_fusion_amd import _lib
    from anchored_fusion_amd.genome import GenomeIndex
    contigs, og, _ = world
    monkeypatch.setenv("AF_G1_HEAVY_EXT", str(max_ext))
    gw = GenomeIndex(contigs, device=0)
    try:
        reads, lens = sample_reads(contigs, 800, seed=50, chimeric=0.4)
        io, no = og.intervals(reads, lens, threads=8)
        ig, ng = gw.intervals(reads, lens)
        _iv_sets_equal(io, no, ig, ng)
        so, sno = og.align_se(reads, lens, id_base=5, threads=8)
        sg, sng = gw.align_se(reads, lens, id_base=5)
        assert np.array_equal(sno, sng)
        for r in range(len(sno)):
            msg = _rec_equal(so[r], sg[r], min(sno[r], 8))
            assert msg is None, (r, msg)
        pairs = sample_pairs(contigs, 500, seed=51)
        plens = np.full(pairs.shape[0], pairs.shape[1], np.int32)
        po, pno = og.align_pe(pairs, plens, pe=oracle.default_pe(chunk_bases=200_000, pair_base=3), threads=8)
        pg, png = gw.align_pe(pairs, plens, pe=_lib.default_pe(chunk_bases=200_000, pair_base=3))
        assert np.array_equal(pno, png)
        for r in range(len(pno)):
            msg = _rec_equal(po[r], pg[r], min(pno[r], 8))
            assert msg is None, (r, msg)
    finally:
        gw.close()


@pytest.mark.parametrize("windows", [1, 3])
def test_pe_rescue_jobs_equal_oracle(world, monkeypatch, windows):
    """S4's heavy pairs (at least AF_G_PE_SPEC_WINDOWS mate-rescue windows, read when the context
    is made): their rescue SWs computed ahead as grid-wide jobs (k_g_pe_jobs), the pair's own walk
    taking the results (k_g_pe mode 2) -- every record equal to the oracle's, on sampled pairs and on
    the crafted rescue pairs of test_genome_rescue_blocks.py."""
    from anchored_fusion_amd import _lib
    from anchored_fusion_amd.genome import GenomeIndex
    from test_genome_rescue_blocks import L, crafted
    contigs, og, _ = world
    monkeypatch.setenv("AF_G_PE_SPEC_WINDOWS", str(windows))
    gj = GenomeIndex(contigs, device=0)
    try:
        pairs = sample_pairs(contigs, 800, seed=61)
        plens = np.full(pairs.shape[0], pairs.shape[1], np.int32)
        po, pno = og.align_pe(pairs, plens, pe=oracle.default_pe(chunk_bases=200_000, pair_base=5), threads=8)
        pg, png = gj.align_pe(pairs, plens, pe=_lib.default_pe(chunk_bases=200_000, pair_base=5))
        assert np.array_equal(pno, png)
        for r in range(len(pno)):
            msg = _rec_equal(po[r], pg[r], min(pno[r], 8))
            assert msg is None, (r, msg)
        assert gj.stats()["pe_rescue_job_pairs"] > 0
    finally:
        gj.close()
    c2, reads, _ = crafted()
    og2 = oracle.OracleGenome(c2)
    g2 = GenomeIndex(c2, device=0)
    try:
        lens = np.full(reads.shape[0], L, np.int32)
        ro, no = og2.align_pe(reads, lens, pe=oracle.default_pe(), pair_base=0, threads=8)
        rg, ng = g2.align_pe(reads, lens, pe=_lib.default_pe())
        assert np.array_equal(no, ng)
        for r in range(len(no)):
            msg = _rec_equal(ro[r], rg[r], min(no[r], 8))
            assert msg is None, (r, msg)
    finally:
        g2.close()
