"""The size-independent bwa-index checks (tests/fm_checks.py, used on the GPU-built 3.09 Gbp
index of configs[2]) on the oracle's index of the repeat-rich test genome: they pass on a correct
index and catch a swapped suffix-array pair, a wrong BWT code and a wrong block count."""
import numpy as np
import pytest

import afpkg  # noqa: F401
import oracle
from fm_checks import check_index, occ_from_sa
from genome_world import make_genome


@pytest.fixture(scope="module")
def index():
    contigs = make_genome(n_ctg=2, ctg_len=(60_000, 40_000), alu_copies=80, young_copies=120, l1_copies=8)
    og = oracle.OracleGenome(contigs)
    T, sa = og.text(), og.sa()
    return og, T, sa, occ_from_sa(T, sa)


def _run(T, sa, occ, og, **kw):
    return check_index(lambda a, n: T[a:a + n], lambda a, n: sa[a:a + n], lambda a, n: occ[a:a + n],
                       og.l_pac, og.primary(), n_rows=300, n_blocks=40, window=64, **kw)


def test_checks_pass_on_the_oracle_index(index):
    og, T, sa, occ = index
    s = _run(T, sa, occ, og)
    assert s["undecided"] == 0 and s["rows"] == 300


def test_checks_catch_a_swapped_pair(index):
    og, T, sa, occ = index
    bad = sa.copy()
    rng = np.random.default_rng(5)
    for r in rng.integers(1, len(sa) - 1, 200):  # many swaps: a sample meets one
        bad[r], bad[r + 1] = bad[r + 1], bad[r]
    with pytest.raises(AssertionError):
        _run(T, bad, occ_from_sa(T, bad), og)


def test_checks_catch_a_wrong_bwt_code_or_count(index):
    og, T, sa, occ = index
    bad = occ.copy()
    bad[5:, 1] += np.uint64(1)  # counts off by one from block 5 on
    with pytest.raises(AssertionError):
        _run(T, sa, bad, og)
    bad = occ.copy()
    bad[:, 4] ^= np.uint64(1)  # the first row's code of every block flipped
    with pytest.raises(AssertionError):
        _run(T, sa, bad, og)


def test_oracle_sais_equals_doubling():
    """The oracle's SA-IS suffix array (linear: tens of Mbp in seconds) equals its prefix-doubling
    construction row for row on random, periodic and duplicated texts."""
    import ctypes
    g = oracle._glib()
    g.afo_suffix_array_check.restype = ctypes.c_int64
    g.afo_suffix_array_check.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    rng = np.random.default_rng(0)
    base = rng.integers(0, 4, 5000).astype(np.uint8)
    cases = [rng.integers(0, k, n).astype(np.uint8) for n in (1, 2, 3, 5, 17, 100, 1000) for k in (1, 2, 4)]
    cases += [np.tile(base[:7], 3000), np.tile(base[:1], 5000),
              np.concatenate([base, base, base[:2000], rng.integers(0, 4, 3000).astype(np.uint8), base])]
    for c in cases:
        c = np.ascontiguousarray(c)
        assert g.afo_suffix_array_check(c.ctypes.data, len(c)) == 0, len(c)
