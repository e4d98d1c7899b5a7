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
