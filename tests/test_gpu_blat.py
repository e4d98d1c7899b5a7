"""GPU BLAT restatement (af_tile_index_build / af_blat, csrc/blat.hip) vs the CPU contract
(oracle/blat.c): every PSL field bit-exact, for each of the reference's option sets."""
import numpy as np
import pytest

import oracle
from oracle_backends import OracleTileReference

pytestmark = pytest.mark.gpu

_B = np.frombuffer(b"ACGT", np.uint8)
_COMP = bytes.maketrans(b"ACGTN", b"TGCAN")


def _world(seed, n_ctg=3, ctg_len=400_000, repeats=True):
    rng = np.random.default_rng(seed)
    ctgs = []
    rep = _B[rng.integers(0, 4, 300)].tobytes()
    for k in range(n_ctg):
        s = bytearray(_B[rng.integers(0, 4, ctg_len)].tobytes())
        if repeats:  # a 300-nt family at ~2 % divergence, 1,500 copies per contig (repMatch, hit caps)
            for _ in range(1500):
                p = int(rng.integers(0, ctg_len - 300))
                c = bytearray(rep)
                for j in np.nonzero(rng.random(300) < 0.02)[0]:
                    c[j] = b"ACGT"[(b"ACGT".index(c[j]) + int(rng.integers(1, 4))) % 4]
                s[p:p + 300] = c
        s[1000:1100] = b"N" * 100
        ctgs.append((f"c{k}", s.decode()))
    return ctgs, rep


def _queries(ctgs, rep, seed, n=600):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = int(rng.integers(0, len(ctgs)))
        g = ctgs[k][1].encode()
        kind = i % 6
        if kind == 0:  # short exact tails (12-40 nt)
            ln = int(rng.integers(12, 41))
            p = int(rng.integers(0, len(g) - ln))
            q = g[p:p + ln]
        elif kind == 1:  # reads with substitutions and an indel
            ln = int(rng.integers(60, 151))
            p = int(rng.integers(0, len(g) - ln - 5))
            q = bytearray(g[p:p + ln])
            for j in np.nonzero(rng.random(ln) < 0.03)[0]:
                q[j] = b"ACGT"[(b"ACGT".index(q[j]) + 1) % 4] if q[j] in b"ACGT" else q[j]
            j = int(rng.integers(10, ln - 10))
            q = bytes(q[:j] + q[j + int(rng.integers(1, 4)):])
        elif kind == 2:  # junction: two parts up to 50 kb apart (a stitched multi-block hit)
            a, b = int(rng.integers(25, 90)), int(rng.integers(25, 90))
            p = int(rng.integers(0, len(g) - 60_000))
            p2 = p + a + int(rng.integers(100, 50_000))
            q = g[p:p + a] + g[p2:p2 + b]
        elif kind == 3:  # reverse strand
            ln = int(rng.integers(20, 200))
            p = int(rng.integers(0, len(g) - ln))
            q = g[p:p + ln][::-1].translate(_COMP)
        elif kind == 4:  # repeat-derived
            q = rep[int(rng.integers(0, 150)):][:int(rng.integers(30, 150))]
        else:  # random
            q = _B[rng.integers(0, 4, int(rng.integers(11, 120)))].tobytes()
        out.append(q.decode())
    return out


def _gpu_ref(ctgs, step):
    from anchored_fusion_amd import blat
    return blat.TileReference(ctgs, step)


PRESETS = ["split_tail", "anchored_split", "genome_validate", "homologs", "candidate_homolog"]


@pytest.mark.parametrize("preset", PRESETS)
def test_blat_parity(preset):
    from anchored_fusion_amd import blat
    ctgs, rep = _world(11)
    qs = _queries(ctgs, rep, 3)
    p = blat.params(preset)
    g = _gpu_ref(ctgs, p.step_size)
    o = OracleTileReference(ctgs, p.step_size)
    rg, ng = g.search(qs, p)
    ro, no = o.search(qs, p)
    assert np.array_equal(ng, no), np.nonzero(ng != no)[0][:10]
    for i in range(len(qs)):
        for k in range(ng[i]):
            a, b = rg[i, k], ro[i, k]
            for f in blat.PSL_DTYPE.names:
                assert np.array_equal(a[f], b[f]), (preset, i, k, f, a[f], b[f])
    assert ng.sum() > 0
    assert g.caps() == o.caps(), preset  # the caps bind for the same query strands
    g.close()


def test_blat_caps_match_oracle():
    """Every cap counter of af_blat_caps (hits, clumps, rows; parts never binds: every clump may
    become a part) on a world where each binds (tests/test_blat_caps.py), equal to the oracle's."""
    from anchored_fusion_amd import blat
    from test_blat_caps import caps_world
    ctgs, qs = caps_world()
    for max_rows in (16, 1):
        p = blat.params("homologs")
        g = _gpu_ref(ctgs, p.step_size)
        o = OracleTileReference(ctgs, p.step_size)
        rg, ng = g.search(qs, p, max_rows)
        ro, no = o.search(qs, p, max_rows)
        assert np.array_equal(ng, no)
        cg, co = g.caps(), o.caps()
        assert cg == co, (max_rows, cg, co)
        assert cg["parts"] == 0 and (min(cg["hits"], cg["clumps"], cg["rows"]) > 0 if max_rows == 1 else cg["hits"] > 0)
        g.close()


def test_blat_query_caps_sum_to_context_caps():
    """af_blat_query_caps: with per-query counters registered, a device search counts every cap
    event per query and none on the context; the per-query counts sum to the context's counts of
    the same search made without them (caps_world, one row slot per query: hits, clumps and rows
    bind)."""
    import torch

    from anchored_fusion_amd import blat
    from anchored_fusion_amd.place import pack_queries
    from test_blat_caps import caps_world
    ctgs, qs = caps_world()
    p = blat.params("homologs")
    g = _gpu_ref(ctgs, p.step_size)
    dev = torch.device("cuda:0")
    buf, lens = pack_queries(qs)
    n = len(qs)
    qt, lt = torch.from_numpy(buf).to(dev), torch.from_numpy(lens).to(dev)
    nq = torch.tensor([n], dtype=torch.int32, device=dev)
    try:
        per = []
        for registered in (False, True):
            rows = torch.zeros(n * blat.MAX_ROWS * blat.PSL_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            nr = torch.zeros(n, dtype=torch.int32, device=dev)
            qc = torch.zeros(4 * n, dtype=torch.int32, device=dev)
            g.caps(reset=True)
            if registered:
                g.query_caps_to(qc, n)
            try:
                g.search_device(qt, nq, buf.shape[1], rows, nr, lens_t=lt, p=p, max_rows=1,
                                stream=torch.cuda.current_stream())
            finally:
                g.query_caps_to()
            torch.cuda.synchronize()
            per.append((g.caps(reset=True), qc.view(4, n).cpu().numpy(), nr.cpu().numpy()))
        (ctx0, _, nr0), (ctx1, qc1, nr1) = per
        assert np.array_equal(nr0, nr1)
        assert all(v == 0 for v in ctx1.values()), ctx1
        assert dict(zip(blat.CAP_NAMES, (int(v) for v in qc1.sum(axis=1)))) == ctx0
        assert ctx0["hits"] > 0 and ctx0["rows"] > 0 and (qc1 > 0).any(axis=0).sum() < n
    finally:
        g.close()


def test_blat_many_parts_equal_oracle():
    """A repeat family of 60 diverged copies and split halves (tests/test_blat_caps.py
    family_world): dozens of parts per query strand, chains across a 2 kb gap, the row cap bound --
    every PSL field and every counter equal to the oracle's, for max_rows 16 and 3."""
    from anchored_fusion_amd import blat
    from test_blat_caps import family_world
    ctgs, qs = family_world()
    rng = np.random.default_rng(4)
    qs = qs + [q[int(a):int(a) + 120] for q, a in zip(qs * 4, rng.integers(0, 100, 8))]
    p = blat.params("split_tail")
    g = _gpu_ref(ctgs, p.step_size)
    o = OracleTileReference(ctgs, p.step_size)
    try:
        for max_rows in (16, 3):
            rg, ng = g.search(qs, p, max_rows)
            hs = g.heavy_stats()
            assert hs["aligned"] == hs["jobs"] and hs["chained"] == hs["deferred"], hs
            ro, no = o.search(qs, p, max_rows)
            assert np.array_equal(ng, no), (max_rows, ng, no, hs)
            for q in range(len(qs)):
                assert rg[q, :ng[q]].tobytes() == ro[q, :no[q]].tobytes(), (max_rows, q)
            cg, co = g.caps(), o.caps()
            assert cg == co and cg["parts"] == 0 and cg["rows"] > 0, (cg, co)
    finally:
        g.close()


def test_blat_finds_what_blat_finds():
    """Behaviours the restatement keeps from BLAT: a 14-15 nt tail places with -stepSize=3
    -minMatch=2 when two tiles fall on it, never with the default step 11; a two-exon read is one
    multi-block hit; -minIdentity drops a diverged hit that -minScore keeps."""
    from anchored_fusion_amd import blat
    ctgs, _ = _world(5, n_ctg=1, repeats=False)
    g = ctgs[0][1]
    ref3, ref11 = _gpu_ref(ctgs, 3), _gpu_ref(ctgs, 11)
    p3 = blat.params("anchored_split")
    t15 = g[3002:3017]  # tiles at 3003 and 3006 (step 3) both inside
    r, n = ref3.search([t15], p3)
    assert n[0] >= 1 and r[0, 0]["t_start"] == 3002 and r[0, 0]["matches"] == 15
    r, n = ref11.search([t15], blat.params("split_tail", min_score=12))
    assert n[0] == 0
    junction = g[50_000:50_070] + g[58_000:58_060]
    r, n = ref11.search([junction], blat.params("split_tail"))
    assert n[0] >= 1 and r[0, 0]["block_count"] == 2 and r[0, 0]["t_num_insert"] == 1
    assert (r[0, 0]["t_start"], r[0, 0]["t_end"]) == (50_000, 58_060)
    diverged = bytearray(g[90_000:90_125].encode())
    for j in range(27, 27 + 6 * 13, 6):  # 13 mismatches: identity 89.6 %
        diverged[j] = b"ACGT"[(b"ACGT".index(diverged[j]) + 1) % 4]
    r, n = ref3.search([diverged.decode()], blat.params("genome_validate"))
    assert n[0] == 0
    r, n = ref3.search([diverged.decode()], blat.params("candidate_homolog"))
    assert n[0] >= 1
    ref3.close()
    ref11.close()


def test_blat_device_matches_host():
    import torch

    from anchored_fusion_amd import blat
    from anchored_fusion_amd.place import pack_queries
    ctgs, rep = _world(2, n_ctg=2)
    qs = _queries(ctgs, rep, 9, n=300)
    p = blat.params("split_tail")
    ref = _gpu_ref(ctgs, p.step_size)
    rh, nh = ref.search(qs, p)
    buf, lens = pack_queries(qs)
    dev = torch.device("cuda:0")
    cap = len(qs) + 17
    qt = torch.zeros((cap, buf.shape[1]), dtype=torch.uint8, device=dev)
    qt[:len(qs)] = torch.from_numpy(buf).to(dev)
    lt = torch.zeros(cap, dtype=torch.int32, device=dev)
    lt[:len(qs)] = torch.from_numpy(lens).to(dev)
    nq = torch.tensor([len(qs)], dtype=torch.int32, device=dev)
    rows = torch.zeros(cap * blat.MAX_ROWS * blat.PSL_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    nr = torch.zeros(cap, dtype=torch.int32, device=dev)
    ref.search_device(qt, nq, buf.shape[1], rows, nr, lens_t=lt, p=p, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    nd = nr[:len(qs)].cpu().numpy()
    rd = rows.cpu().numpy().view(blat.PSL_DTYPE).reshape(cap, blat.MAX_ROWS)[:len(qs)]
    assert np.array_equal(nd, nh)
    for i in range(len(qs)):
        assert rd[i, :nd[i]].tobytes() == rh[i, :nh[i]].tobytes()
    ref.close()


def test_blat_tile_index_from_device_matches_host():
    import torch

    from anchored_fusion_amd import blat
    from anchored_fusion_amd.place import concat_contigs
    ctgs, rep = _world(4, n_ctg=2)
    blob, offs = concat_contigs(ctgs)
    bt = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda()
    a = blat.TileReference.from_device(bt, [n for n, _ in ctgs], [len(s) for _, s in ctgs], offs, 3)
    b = _gpu_ref(ctgs, 3)
    qs = _queries(ctgs, rep, 1, n=120)
    p = blat.params("anchored_split")
    ra, na = a.search(qs, p)
    rb, nb = b.search(qs, p)
    assert np.array_equal(na, nb) and ra.tobytes() == rb.tobytes()


@pytest.mark.gpu
def test_blat_device_range_matches_host():
    """af_blat_device_range: queries [first, n) only, rows at their own indices; the rest of the
    output untouched."""
    import torch

    from anchored_fusion_amd import blat
    from anchored_fusion_amd.place import pack_queries
    ctgs, rep = _world(3, n_ctg=2)
    qs = _queries(ctgs, rep, 11, n=200)
    p = blat.params("split_tail")
    ref = _gpu_ref(ctgs, p.step_size)
    rh, nh = ref.search(qs, p)
    buf, lens = pack_queries(qs)
    dev = torch.device("cuda:0")
    qt = torch.from_numpy(buf).to(dev)
    lt = torch.from_numpy(lens).to(dev)
    nq = torch.tensor([len(qs)], dtype=torch.int32, device=dev)
    first = torch.tensor([77], dtype=torch.int32, device=dev)
    rows = torch.zeros(len(qs) * blat.MAX_ROWS * blat.PSL_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    nr = torch.full((len(qs),), -5, dtype=torch.int32, device=dev)
    ref.search_device(qt, nq, buf.shape[1], rows, nr, lens_t=lt, p=p, stream=torch.cuda.current_stream(),
                      first_t=first)
    torch.cuda.synchronize()
    nd = nr.cpu().numpy()
    rd = rows.cpu().numpy().view(blat.PSL_DTYPE).reshape(len(qs), blat.MAX_ROWS)
    assert (nd[:77] == -5).all()
    assert np.array_equal(nd[77:], nh[77:])
    for i in range(77, len(qs)):
        assert rd[i, :nd[i]].tobytes() == rh[i, :nh[i]].tobytes()
    ref.close()


def test_blat_edge_cases():
    """Empty and sub-tile queries, all-N, the maximum length (AF_MAX_READ), queries across the
    N run and at contig ends, a query set of one, and no queries: GPU == oracle, field by field."""
    from anchored_fusion_amd import _lib, blat
    ctgs, rep = _world(5, n_ctg=2, ctg_len=200_000)
    g0 = ctgs[0][1]
    qs = ["", "A", "ACGTACGTAC", "N" * 60, g0[900:1000] + g0[1100:1180],  # the N run cut out: a junction
          g0[950:1150],                                                 # across the N run
          g0[:70], g0[-90:], g0[5000:5000 + _lib.AF_MAX_READ],           # contig ends, the maximum length
          rep[:_lib.AF_MAX_READ // 2] * 2, g0[7000:7011]]               # repeat-heavy, exactly one tile
    for preset in ("split_tail", "anchored_split"):
        p = blat.params(preset)
        g = _gpu_ref(ctgs, p.step_size)
        o = OracleTileReference(ctgs, p.step_size)
        for batch in (qs, qs[8:9]):
            rg, ng = g.search(batch, p)
            ro, no = o.search(batch, p)
            assert np.array_equal(ng, no), (preset, ng, no)
            for i in range(len(batch)):
                assert rg[i, :ng[i]].tobytes() == ro[i, :no[i]].tobytes(), (preset, i)
        rg, ng = g.search([], p)
        assert len(ng) == 0
        g.close()


def test_blat_spill_rows_equal_oracle_all_rows():
    """Rows past MAX_ROWS (af_blat_spill; TileReference.search_all, every BLAT call of the Placer
    and S6): the kept rows followed by the spilled ones in row order equal the oracle's full row
    list (max_rows 256), field by field; nothing is counted as dropped."""
    from anchored_fusion_amd import blat
    from test_blat_caps import family_world
    ctgs, qs = family_world()
    rng = np.random.default_rng(8)
    qs = qs + [q[int(a):int(a) + 150] for q, a in zip(qs * 3, rng.integers(0, 80, 6))]
    p = blat.params("split_tail")
    g = _gpu_ref(ctgs, p.step_size)
    o = OracleTileReference(ctgs, p.step_size)
    try:
        g.caps()
        rows, nr, extra = g.search_all(qs, p)
        ro, no = o.search(qs, p, 256)
        assert g.caps()["rows"] == 0
        assert (no > blat.MAX_ROWS).sum() >= 2 and (no < 256).all()
        for q in range(len(qs)):
            got = [rows[q, k] for k in range(nr[q])] + extra.get(q, [])
            assert len(got) == no[q], (q, len(got), no[q])
            for k, r in enumerate(got):
                assert r.tobytes() == ro[q, k].tobytes(), (q, k)
    finally:
        g.close()


@pytest.mark.parametrize("heavy", ["1", "0"])
def test_blat_heavy_jobs_equal_oracle(monkeypatch, heavy):
    """A strand with more than AF_BLAT_HEAVY_CLUMPS clumps is deferred (its clumps aligned as
    grid-wide jobs by k_blat_jobs, its chains by k_blat_heavy): with every multi-clump strand
    deferred (1) and with none (0), the device search equals the oracle -- rows, spilled rows, caps
    (family_world: dozens of parts per strand; _world: the parity queries)."""
    import torch

    from anchored_fusion_amd import blat
    from test_blat_caps import family_world
    monkeypatch.setenv("AF_BLAT_HEAVY_CLUMPS", heavy)
    for ctgs, qs, preset in ((family_world()[0], family_world()[1], "split_tail"),
                             (_world(11)[0], _queries(*_world(11), 3, n=60), "anchored_split")):
        p = blat.params(preset)
        g = _gpu_ref(ctgs, p.step_size)
        o = OracleTileReference(ctgs, p.step_size)
        try:
            rg, ng, eg = g.search_all(qs, p, spill_cap=1 << 17)
            ro, no = o.search(qs, p, 4096)  # every row of a query
            assert (no < 4096).all()
            assert np.array_equal(no, ng + np.array([len(eg.get(i, [])) for i in range(len(qs))]))
            for i in range(len(qs)):
                mine = [r.tobytes() for r in rg[i, :min(int(ng[i]), blat.MAX_ROWS)]] + \
                       sorted(r.tobytes() for r in eg.get(i, []))
                theirs = [r.tobytes() for r in ro[i, :min(int(ng[i]), blat.MAX_ROWS)]] + \
                         sorted(r.tobytes() for r in ro[i, blat.MAX_ROWS:no[i]])
                assert mine == theirs, (preset, i)
            cg, co = g.caps(), o.caps()
            assert cg["hits"] == co["hits"] and cg["clumps"] == co["clumps"] and cg["parts"] == co["parts"]
        finally:
            g.close()
        torch.cuda.synchronize()


def test_blat_begin_end_live_mask():
    """af_blat_device_begin / _end with a live mask (the S6 search beside S5): the live queries'
    rows equal a whole search's, the others get none -- heavy strands included (every strand with
    more than one clump deferred)."""
    import os

    import torch

    from anchored_fusion_amd import blat
    from anchored_fusion_amd.place import pack_queries
    from test_blat_caps import family_world
    os.environ["AF_BLAT_HEAVY_CLUMPS"] = "1"
    try:
        ctgs, qs = family_world()
        p = blat.params("split_tail")
        g = _gpu_ref(ctgs, p.step_size)
    finally:
        del os.environ["AF_BLAT_HEAVY_CLUMPS"]
    dev = torch.device("cuda:0")
    buf, lens = pack_queries(qs)
    n = len(qs)
    qt, lt = torch.from_numpy(buf).to(dev), torch.from_numpy(lens).to(dev)
    nq = torch.tensor([n], dtype=torch.int32, device=dev)
    live = torch.from_numpy((np.arange(n) % 3 != 1).astype(np.uint8)).to(dev)
    try:
        rows_a = torch.zeros(n * blat.MAX_ROWS * blat.PSL_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        nr_a = torch.zeros(n, dtype=torch.int32, device=dev)
        g.search_device(qt, nq, buf.shape[1], rows_a, nr_a, lens_t=lt, p=p, stream=torch.cuda.current_stream())
        rows_b = torch.zeros_like(rows_a)
        nr_b = torch.full((n,), 7, dtype=torch.int32, device=dev)
        g.search_device_begin(qt, nq, buf.shape[1], rows_b, nr_b, lens_t=lt, p=p, stream=torch.cuda.current_stream())
        g.search_device_end(live, stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        ra = rows_a.cpu().numpy().view(blat.PSL_DTYPE).reshape(n, blat.MAX_ROWS)
        rb = rows_b.cpu().numpy().view(blat.PSL_DTYPE).reshape(n, blat.MAX_ROWS)
        na, nb, lv = nr_a.cpu().numpy(), nr_b.cpu().numpy(), live.cpu().numpy()
        assert na[lv == 1].sum() > 0
        for i in range(n):
            if lv[i]:
                assert nb[i] == na[i] and ra[i, :na[i]].tobytes() == rb[i, :nb[i]].tobytes(), i
            else:
                assert nb[i] == 0, i
    finally:
        g.close()
