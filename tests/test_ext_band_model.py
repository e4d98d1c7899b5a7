"""The lane layout of ksw_dp.h's ext_dp_band (the diagonal band kernel BLAT's clump extensions
run), restated lane by lane in Python (64 lanes, lane k = column i - w + k of row i: the DPP
prefix max and one-lane shifts as list operations), checked on the CPU against the oracle's
ksw_extend2 (oracle/af_oracle.c afo_ext_dp): max, qle, tle, gtle, gscore and max_off on random
cases with bands 0-31, BLAT's and bwa's scores, h0 up to 250, z-drop off / tight and N bases.
The kernel itself is held to the oracle on the GPU by tests/test_gpu_ext_dp.py."""
import ctypes
import random

import oracle

NEG = -(1 << 31)


def div_plus(x, y, c):
    return x + c if y == 1 else int(x / y + c)


def incl_max(v):
    """Inclusive prefix max over the 64 lanes (the kernel's DPP scan)."""
    out, c = [], NEG
    for x in v:
        c = max(c, x)
        out.append(c)
    return out


def band(qlen, q, tlen, t, a, b, od, ed, oi, ei, w, end_bonus, zdrop, h0, exitmask=3):
    """ext_dp_band's rows: lists of 64 lane values, lane k = column i - w + k of row i."""
    oe_del, oe_ins = od + ed, oi + ei
    w = min(w, max(div_plus(qlen * a + end_bonus - oi, ei, 1), 1))
    w = min(w, max(div_plus(qlen * a + end_bonus - od, ed, 1), 1))
    assert w <= 31
    v1 = h0 - oe_ins if h0 > oe_ins else 0
    lanes = range(64)

    def h_init(j):
        return 0 if j < 0 or j > qlen else (h0 if j == 0 else max(v1 - (j - 1) * ei, 0))

    J = [k - w for k in lanes]
    H = [h_init(j) for j in J]
    E = [0] * 64
    tail = [k >= 2 * w + 1 for k in lanes]
    mx, max_i, max_j, max_ie, gscore, max_off = h0, -1, -1, -1, -1, 0
    beg, end = 0, qlen
    for i in range(tlen):
        ti = t[i]
        qc = [q[j] if 0 <= j < qlen else 4 for j in J]
        beg = max(beg, i - w)
        end = min(end, i + w + 1, qlen)
        h1s = max(h0 - (od + ed * (i + 1)), 0) if beg == 0 else 0
        if beg >= end:
            if beg == qlen:
                max_ie = max_ie if gscore > h1s else i
                gscore = max(gscore, h1s)
            break
        inb = [beg <= j < end for j in J]
        s_eq, s_ne = (-1, -1) if ti > 3 else (a, -b)
        M = []
        for k in lanes:
            sc = s_eq if qc[k] == ti else (-1 if qc[k] > 3 else s_ne)
            M.append((H[k] + sc if H[k] != 0 else 0) if inb[k] else 0)
        jE = [j * ei for j in J]
        jE1 = [(1 << 30) if j <= 0 else j * ei - ei for j in J]
        P = [0] + incl_max([max(M[k] + jE[k] - oe_ins, jE[k]) for k in lanes])[:-1]  # shr 1, 0 into lane 0
        h = [max(M[k], E[k], P[k] - jE1[k]) for k in lanes]
        keys = [(h[k] << 10 | J[k]) if inb[k] else -1 for k in lanes]
        kmax = max(keys)
        m, mj = max(kmax, 0) >> 10, (-1 if kmax < 0 else kmax & 1023)
        hq = h[min(max(qlen - 1 - i + w, 0), 63)]
        Eu = [max(E[k] - ed, M[k] - oe_del, 0) for k in lanes]
        En = [Eu[k] if J[k] < end else (0 if J[k] == end else E[k]) for k in lanes]
        e_beg = En[0]
        Hs, Es = H[1:] + [0], En[1:] + [0]  # shl 1, 0 into lane 63
        Jn = [j + 1 for j in J]
        H = [h1s if Jn[k] == beg else (h[k] if Jn[k] <= end else Hs[k]) for k in lanes]
        E = Es
        for k in lanes:
            if tail[k]:
                H[k], E[k] = (0 if Jn[k] > qlen else max(v1 - (Jn[k] - 1) * ei, 0)), 0
        if end == qlen:
            max_ie = max_ie if gscore > hq else i
            gscore = max(gscore, hq)
        better = m > mx
        di, dj = i - max_i, mj - max_j
        zgap = mx - m - (di - dj) * ed if di > dj else mx - m - (dj - di) * ei
        if better:
            max_off, max_i, max_j, mx = max(max_off, abs(mj - i)), i, mj, m
        if m == 0 or (not better and zdrop > 0 and zgap > zdrop):
            break
        x = [(Jn[k] - beg) if (H[k] | E[k]) != 0 else (1 << 20) for k in lanes]
        fm = [k for k in lanes if 0 <= x[k] < end - beg]
        lm = [k for k in lanes if 0 <= x[k] <= end - beg]
        edge = beg == i - w and (h1s | e_beg) != 0  # column i - w: no lane in the next row
        c0 = i + 1 - w
        beg_new = beg if edge else (c0 + fm[0] if fm else end)
        lnz = c0 + lm[-1] if lm else (beg if edge else -1)
        jstar = lnz if lnz >= beg_new else beg_new - 1
        beg, end = beg_new, min(jstar + 2, qlen)
        J = Jn
        if (i & exitmask) == exitmask:
            U = max(max(H[k], E[k]) + (qlen - J[k]) * a if 0 <= J[k] - beg <= qlen - beg else 0 for k in lanes)
            if U <= mx and U < gscore and gscore > 0:
                break
    return (mx, max_j + 1, max_i + 1, max_ie + 1, gscore, max_off)


def _oracle(q, t, a, b, od, ed, oi, ei, w, end_bonus, zdrop, h0):
    import numpy as np
    L = oracle.lib()
    L.afo_ext_dp.restype = ctypes.c_int
    L.afo_ext_dp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                             ctypes.POINTER(oracle.Params), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int] + \
        [ctypes.POINTER(ctypes.c_int)] * 5
    p = oracle.default_params()
    p.a, p.b, p.o_del, p.e_del, p.o_ins, p.e_ins = a, b, od, ed, oi, ei
    r = [ctypes.c_int() for _ in range(5)]
    qa = np.array(q, np.uint8)
    ta = np.array(t, np.uint8)
    mx = L.afo_ext_dp(len(q), qa.ctypes.data, len(t), ta.ctypes.data, ctypes.byref(p), w, end_bonus, zdrop, h0,
                      *[ctypes.byref(x) for x in r])
    return (mx,) + tuple(x.value for x in r)


def test_band_layout_model_equals_oracle():
    rnd = random.Random(7)
    n = 0
    for _ in range(800):
        qlen = rnd.randint(64, 200)
        q = [rnd.randrange(4) for _ in range(qlen)]
        if rnd.random() < 0.1:
            q = [x if rnd.random() > 0.02 else 4 for x in q]
        w = rnd.choice([16, 16, 16, 8, 31, 20, 3, 0, 1])
        tlen = rnd.randint(1, qlen + w + 5)
        t, k = [], 0
        while len(t) < tlen:
            r = rnd.random()
            if k < qlen and r < 0.9:
                t.append(q[k] if rnd.random() > 0.03 else rnd.randrange(5))
                k += 1
            elif r < 0.93:
                k += rnd.randint(1, 3)
            elif r < 0.96:
                t.append(rnd.randrange(4))
            else:
                t.append(rnd.randrange(4))
                k += 1
        h0 = rnd.choice([11, 1, 5, 30, 150, 250, rnd.randint(1, 200)])
        a, b, od, ed, oi, ei = (1, 1, 3, 1, 3, 1) if rnd.random() < 0.7 else (1, 4, 6, 1, 6, 1)
        zd = rnd.choice([20, 100, 0, 5])
        got = band(qlen, q, tlen, t, a, b, od, ed, oi, ei, w, 0, zd, h0)
        want = _oracle(q, t, a, b, od, ed, oi, ei, w, 0, zd, h0)
        assert got == want, (qlen, tlen, w, h0, zd, got, want)
        n += 1
    assert n == 800
