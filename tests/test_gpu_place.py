"""GPU parity of the placement kernel (af_place, K2 in multi-hit mode) against the oracle
(afo_place): every hit field bit-exact, best-first order included."""
import numpy as np
import pytest

import afpkg  # noqa: F401
import oracle
from anchored_fusion_amd import place
from place_cases import contigs, queries

pytestmark = pytest.mark.gpu


def _same(g, gn, r, rn):
    assert np.array_equal(gn, rn)
    for i in range(len(gn)):
        for k in range(max(int(gn[i]), 0)):
            a, b = g[i, k], r[i, k]
            for f in ("query", "flag", "score", "q_start", "q_end", "q_size", "matches", "n_cigar", "t_start",
                      "t_end"):
                assert a[f] == b[f], (i, k, f, a[f], b[f])
            assert np.array_equal(a["cigar"], b["cigar"]), (i, k)


@pytest.mark.parametrize("T,seed_len,max_hits,lens", [(20, 16, 8, (20, 40, 60, 100, 150)),
                                                      (30, 19, 4, (100, 150, 250)),
                                                      (12, 16, 16, (16, 18, 25, 33))])
def test_place_parity(T, seed_len, max_hits, lens):
    ctgs = contigs(seed=T)
    blob, _ = place.concat_contigs(ctgs)
    qs = queries(ctgs, 1500, seed=T + 1, lens=lens)
    seqs = [q for _, q, _ in qs]
    ref = place.Reference(ctgs)
    p = place._lib.default_params()
    p.T, p.min_seed_len = T, seed_len
    g, gn = ref.raw_hits(seqs, p, max_hits)
    buf, ln = place.pack_queries(seqs)
    po = oracle.default_params()
    po.T, po.min_seed_len = T, seed_len
    r, rn = oracle.OracleIndex(blob).place(buf, ln, po, max_hits, threads=8)
    _same(g, gn, r, rn)
    assert (gn > 0).sum() > 0.5 * len(qs)
    ref.close()


def test_placer_psl_rows():
    ctgs = contigs(n=3, length=6000)
    qs = queries(ctgs, 200, seed=3, lens=(60, 100))
    pl = place.Placer()
    rows = pl(ctgs, [(n, q) for n, q, _ in qs], "split_tail")
    body = [r.split("\t") for r in rows if r[:1].isdigit()]
    assert body and all(len(f) == 21 for f in body)
    names = {n for n, _ in ctgs}
    for f in body:
        assert f[13] in names and 0 <= int(f[15]) < int(f[16]) <= int(f[14])
        assert 0 <= int(f[11]) < int(f[12]) <= int(f[10])
    pl.close()


def _repeat_contigs(seed=5):
    """Contigs with exact repeats on both strands, a palindromic 16-mer run and N runs: 16-mers
    whose occurrences mix forward and reverse-strand images (the genome index adds the latter
    from the reverse complement's forward run)."""
    from place_cases import rc
    rng = np.random.default_rng(seed)
    base = "".join(rng.choice(list("ACGT"), 9000))
    unit = base[1000:1400]
    pal = "ACGTTGCAACGTTGCA" * 3  # rc(pal) == pal
    c1 = base[:3000] + unit + base[3000:5000] + rc(unit) + "N" * 40 + base[5000:7000] + pal + base[7000:]
    c2 = "".join(rng.choice(list("ACGT"), 12000))
    c2 = c2[:4000] + unit + c2[4000:8000] + rc(c1[200:500]) + c2[8000:]
    return [("chrA", c1), ("chrB", c2)]


@pytest.mark.parametrize("case", ["random", "repeats"])
def test_place_parity_genome_index(monkeypatch, case):
    # the GPU-built direct 16-mer table (af_index_build_genome) gives the same hits as the oracle
    monkeypatch.setenv("AF_INDEX_KIND", "genome")
    ctgs = contigs(seed=3) if case == "random" else _repeat_contigs()
    blob, _ = place.concat_contigs(ctgs)
    qs = queries(ctgs, 1200, seed=9, lens=(20, 40, 60, 100, 150))
    if case == "repeats":
        qs += [("u", ctgs[0][1][2990:3100], None), ("p", "TT" + "ACGTTGCAACGTTGCA" * 3 + "GG", None)]
    seqs = [q for _, q, _ in qs]
    ref = place.Reference(ctgs)
    assert ref.kind == "genome"
    for T, seed_len in ((20, 16), (30, 19)):
        p = place._lib.default_params()
        p.T, p.min_seed_len = T, seed_len
        g, gn = ref.raw_hits(seqs, p, 8)
        buf, ln = place.pack_queries(seqs)
        po = oracle.default_params()
        po.T, po.min_seed_len = T, seed_len
        r, rn = oracle.OracleIndex(blob).place(buf, ln, po, 8, threads=8)
        _same(g, gn, r, rn)
    ref.close()


def test_genome_index_large_reference():
    # 320 Mbp in 4 contigs (auto-selects the genome index): reads drawn from known positions,
    # half reverse-complemented, are placed there (no oracle at this size)
    from place_cases import rc
    rng = np.random.default_rng(17)
    lens = (80_000_000,) * 4
    ctgs = [(f"chr{k + 1}", rng.choice(np.frombuffer(b"ACGT", np.uint8), n).tobytes().decode())
            for k, n in enumerate(lens)]
    ref = place.Reference(ctgs)
    assert ref.kind == "genome"
    seqs, truth = [], []
    for i in range(2000):
        k = int(rng.integers(4))
        s = int(rng.integers(0, lens[k] - 150))
        q = ctgs[k][1][s:s + 150]
        rev = i % 2 == 1
        seqs.append(rc(q) if rev else q)
        truth.append((k, s, rev))
    p = place._lib.default_params()
    g, gn = ref.raw_hits(seqs, p, 4)
    ok = 0
    for i, (k, s, rev) in enumerate(truth):
        if gn[i] < 1:
            continue
        h = g[i, 0]
        loc = ref.locate(h["t_start"], h["t_end"])
        ok += loc is not None and loc[0] == k and loc[1] == s and bool(h["flag"] & 0x10) == rev and h["score"] == 150
    assert ok == len(truth)
    ref.close()


@pytest.mark.parametrize("kind", ["hash", "genome"])
def test_place_reseed_on_mem_overflow(monkeypatch, kind):
    """Queries with more than max_mems MEMs at the minimum length: twelve diverged copies of a
    2 kb unit (a substitution every 18 bases, so the copies share many 16-mers but few 20-mers)
    plus one exact source.  The placement re-seeds with the minimum MEM length raised (+4 at a
    time) until at most max_mems MEMs remain; GPU and oracle agree and the exact source wins."""
    monkeypatch.setenv("AF_INDEX_KIND", kind)
    rng = np.random.default_rng(61)
    unit = rng.choice(list("ACGT"), 2000)
    parts = ["".join(rng.choice(list("ACGT"), 3000))]
    for _ in range(12):
        u = unit.copy()
        for i in range(int(rng.integers(0, 18)), len(u), 18):
            u[i] = "ACGT"[("ACGT".index(u[i]) + int(rng.integers(1, 4))) % 4]
        parts += ["".join(u), "".join(rng.choice(list("ACGT"), 500))]
    src = 3000 + 12 * 2500
    parts += ["".join(unit), "".join(rng.choice(list("ACGT"), 3000))]
    ctgs = [("rep", "".join(parts))]
    blob, _ = place.concat_contigs(ctgs)
    seqs = ["".join(unit[s:s + 90]) for s in range(0, 1800, 37)]
    ref = place.Reference(ctgs)
    assert ref.kind == kind
    p = place._lib.default_params()
    p.T, p.min_seed_len = 20, 16
    g, gn = ref.raw_hits(seqs, p, 4)
    buf, ln = place.pack_queries(seqs)
    po = oracle.default_params()
    po.T, po.min_seed_len = 20, 16
    r, rn = oracle.OracleIndex(blob).place(buf, ln, po, 4, threads=8)
    _same(g, gn, r, rn)
    # without re-seeding these queries would overflow (12 copies x ~40 shared 16-mers > 64)
    assert (gn > 0).all()
    for i, s in enumerate(range(0, 1800, 37)):
        assert g[i, 0]["t_start"] == src + s and g[i, 0]["score"] == 90
    ref.close()
