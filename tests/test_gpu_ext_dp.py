"""ksw_extend2 on the GPU (ksw_dp.h ext_dp: the column-per-lane kernels and, when the clamped
band fits the wave and the query does not, the diagonal band layout ext_dp_band) against the
oracle's restatement (oracle/af_oracle.c afo_ext_dp, bwa 0.7.17 ksw_extend2) field by field:
max, qle, tle, gtle, gscore, max_off.  Cases cover every dispatch (qlen 1..320, bands 0..31
and 50 / 100), BLAT's scores (1 / 1 / 3+1, band 16, z-drop 20) and bwa's (1 / 4 / 6+1), h0
from 1 to 250 (a right extension starts from the left one's score), z-drop off / tight,
end bonus, N bases, and targets that are the query with substitutions and indels, a random
tail past a junction, or unrelated sequence.  Through the test hook af_debug_ext_dp (blat.hip,
not part of afgpu.h)."""
import ctypes

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

STRIDE = 1024


def _cases(seed, n):
    rng = np.random.default_rng(seed)
    qs, ts, par = [], [], []
    for k in range(n):
        qlen = int(rng.choice([int(rng.integers(1, 64)), int(rng.integers(64, 128)), int(rng.integers(128, 321))]))
        q = rng.integers(0, 4, qlen).astype(np.uint8)
        if rng.random() < 0.1:
            q[rng.random(qlen) < 0.02] = 4
        w = int(rng.choice([16, 16, 16, 0, 1, 3, 8, 20, 31, 50, 100]))
        kind = rng.random()
        t = []
        i = 0
        tl = int(rng.integers(1, min(STRIDE, qlen + w + 40)))
        while len(t) < tl:
            r = rng.random()
            if kind < 0.15:  # unrelated
                t.append(int(rng.integers(0, 4)))
            elif i < qlen and r < 0.9:
                b = int(q[i]) if rng.random() > 0.03 else int(rng.integers(0, 5))
                t.append(min(b, 4))
                i += 1
            elif r < 0.94:
                i += int(rng.integers(1, 4))  # deletion from the target
            elif r < 0.97:
                t.append(int(rng.integers(0, 4)))  # insertion into the target
            else:
                t.append(int(rng.integers(0, 4)))
                i += 1
            if kind > 0.85 and i > qlen // 2:  # a junction: random past the middle
                kind = 0.0
        blat = rng.random() < 0.6
        a, b, od, ed, oi, ei = (1, 1, 3, 1, 3, 1) if blat else (1, 4, 6, 1, 6, 1)
        zdrop = int(rng.choice([20, 100, 0, 5]))
        end_bonus = int(rng.choice([0, 0, 5]))
        h0 = int(rng.choice([11, 1, 5, 30, 100, 150, 250, int(rng.integers(1, 200))]))
        qs.append(q)
        ts.append(np.array(t, np.uint8))
        par.append([a, b, od, ed, oi, ei, w, end_bonus, zdrop, h0])
    return qs, ts, np.array(par, np.int32)


def _gpu(qs, ts, par):
    from anchored_fusion_amd import _lib
    L = _lib.lib()
    L.af_debug_ext_dp.restype = ctypes.c_int
    L.af_debug_ext_dp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    n = len(qs)
    qb = np.zeros((n, STRIDE), np.uint8)
    tb = np.zeros((n, STRIDE), np.uint8)
    for k in range(n):
        qb[k, :len(qs[k])] = qs[k]
        tb[k, :len(ts[k])] = ts[k]
    ql = np.array([len(x) for x in qs], np.int32)
    tl = np.array([len(x) for x in ts], np.int32)
    out = np.zeros((n, 7), np.int32)
    assert L.af_debug_ext_dp(qb.ctypes.data, tb.ctypes.data, STRIDE, ql.ctypes.data, tl.ctypes.data,
                             par.ctypes.data, n, out.ctypes.data) == 0
    return out


def _oracle(q, t, c):
    L = oracle.lib()
    L.afo_ext_dp.restype = ctypes.c_int
    L.afo_ext_dp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                             ctypes.POINTER(oracle.Params), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int] + \
        [ctypes.POINTER(ctypes.c_int)] * 5
    p = oracle.default_params()
    p.a, p.b, p.o_del, p.e_del, p.o_ins, p.e_ins = (int(x) for x in c[:6])
    r = [ctypes.c_int() for _ in range(5)]
    q = np.ascontiguousarray(q)
    t = np.ascontiguousarray(t) if len(t) else np.zeros(1, np.uint8)
    mx = L.afo_ext_dp(len(q), q.ctypes.data, len(t) if t.size and len(t) else 0, t.ctypes.data, ctypes.byref(p),
                      int(c[6]), int(c[7]), int(c[8]), int(c[9]), *[ctypes.byref(x) for x in r])
    return [mx] + [x.value for x in r]


@pytest.mark.parametrize("seed", [1, 2])
def test_ext_dp_equals_oracle(seed):
    qs, ts, par = _cases(seed, 1500)
    out = _gpu(qs, ts, par)
    bad = []
    for k in range(len(qs)):
        want = _oracle(qs[k], ts[k], par[k])
        got = out[k, :6].tolist()
        if got != want:
            bad.append((k, len(qs[k]), len(ts[k]), par[k].tolist(), got, want))
    assert not bad, bad[:5]


def test_ext_dp_band_layout_is_exercised():
    """The band-layout dispatch condition holds for BLAT's 150-nt extensions (qlen >= 64, w = 16
    after the clamp) -- the cases above include them by construction."""
    qs, ts, par = _cases(1, 1500)
    n_band = sum(1 for q, c in zip(qs, par) if len(q) >= 64 and c[6] <= 31)
    assert n_band > 300
