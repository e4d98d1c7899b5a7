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


def incl_max(v):  # full-wave inclusive prefix max
    out=[];c=NEG
    for x in v: c=max(c,x); out.append(c)
    return out
def band(qlen,q,tlen,t,a,b,od,ed,oi,ei,w,end_bonus,zdrop,h0,exitmask=3):
    oe_del=od+ed; oe_ins=oi+ei
    mi=max(div_plus(qlen*a+end_bonus-oi,ei,1),1); w=min(w,mi)
    md=max(div_plus(qlen*a+end_bonus-od,ed,1),1); w=min(w,md)
    assert w<=31
    v1=h0-oe_ins if h0>oe_ins else 0
    L=range(64)
    J=[k-w for k in L]
    def hinit(j): return 0 if j<0 or j>qlen else (h0 if j==0 else max(v1-(j-1)*ei,0))
    H=[hinit(j) for j in J]; E=[0]*64
    tail=[k>=2*w+1 for k in L]
    mx=h0; max_i=max_j=max_ie=gscore=-1; max_off=0
    beg=0; end=qlen
    def qat(j): return q[min(max(j,0),qlen-1)]
    for i in range(tlen):
        ti=t[i]
        qc=[qat(j) if 0<=j<qlen else 4 for j in J]
        beg=max(beg,i-w); end=min(end,i+w+1,qlen)
        h1s=max(h0-(od+ed*(i+1)),0) if beg==0 else 0
        if beg>=end:
            if beg==qlen:
                max_ie = max_ie if gscore>h1s else i
                gscore=max(gscore,h1s)
            break
        inb=[beg<=j<end for j in J]
        s_eq=-1 if ti>3 else a; s_ne=-1 if ti>3 else -b
        M=[]
        for k in L:
            sc=s_eq if qc[k]==ti else (-1 if qc[k]>3 else s_ne)
            mm=H[k]+sc if H[k]!=0 else 0
            M.append(mm if inb[k] else 0)
        jE=[j*ei for j in J]; jEo=[x-oe_ins for x in jE]; jE1=[(1<<30) if j<=0 else j*ei-ei for j in J]
        run=[max(M[k]+jEo[k],jE[k]) for k in L]
        pm=incl_max(run); P=[0]+pm[:-1]
        f=[P[k]-jE1[k] for k in L]
        h=[max(M[k],E[k],f[k]) for k in L]
        keys=[(h[k]<<10|J[k]) if inb[k] else -1 for k in L]
        kmax=max(keys); m=max(kmax,0)>>10; mj=-1 if kmax<0 else kmax&1023
        hq=h[min(max(qlen-1-i+w,0),63)]
        Eu=[max(E[k]-ed,M[k]-oe_del,0) for k in L]
        En=[Eu[k] if J[k]<end else (0 if J[k]==end else E[k]) for k in L]
        e_beg=En[0]
        Hs=H[1:]+[0]; Es=En[1:]+[0]
        Jn=[j+1 for j in J]
        H=[h1s if Jn[k]==beg else (h[k] if Jn[k]<=end else Hs[k]) for k in L]
        E=Es[:]
        for k in L:
            if tail[k]:
                H[k]=0 if Jn[k]>qlen else max(v1-(Jn[k]-1)*ei,0); E[k]=0
        if end==qlen:
            max_ie = max_ie if gscore>hq else i
            gscore=max(gscore,hq)
        better=m>mx
        di=i-max_i; dj=mj-max_j
        zgap = mx-m-(di-dj)*ed if di>dj else mx-m-(dj-di)*ei
        if better:
            max_off=max(max_off,abs(mj-i)); max_i=i; max_j=mj; mx=m
        stop = 1 if m==0 else (zdrop if (not better and zgap>zdrop) else 0)
        if stop>0: break
        x=[(Jn[k]-beg) if (H[k]|E[k])!=0 else (1<<20) for k in L]
        fm=[k for k in L if 0<=x[k]<end-beg]; lm=[k for k in L if 0<=x[k]<=end-beg]
        edge = beg==i-w and (h1s|e_beg)!=0
        c0=i+1-w
        beg_new = beg if edge else (c0+fm[0] if fm else end)
        lnz = c0+lm[-1] if lm else (beg if edge else -1)
        jstar = lnz if lnz>=beg_new else beg_new-1
        beg=beg_new; end = jstar+2 if jstar+2<qlen else qlen
        J=Jn
        if (i&exitmask)==exitmask:
            u=[max(H[k],E[k])+(qlen-J[k])*a if 0<=J[k]-beg<=qlen-beg else 0 for k in L]
            U=max(u)
            if U<=mx and U<gscore and gscore>0: break
    return (mx,max_j+1,max_i+1,max_ie+1,gscore,max_off)



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
    for _ in range(160):
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
    assert n == 160
