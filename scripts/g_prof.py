"""Per-read profile of the genome calls of one configs[2] step on the profiling build
libafgpu_gprof.so (make -C anchored-fusion_amd/csrc gprof; AF_GPU_LIB=libafgpu_gprof.so).

Prints, per call, the distribution of G1 (k_g_seeds) and G2 (k_g_regions) cycles per read, the
G2 phase shares (mem_chain, chain filter, chain2aln, dedup/patch), the heaviest reads with their
interval / occurrence / chain / region counts, and the G2 schedule (per-wave busy time vs the
makespan).
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("AF_GPU_LIB", "libafgpu_gprof.so")
# one genome call for S4 and S5 (their split into two concurrent calls would share the profile slot)
os.environ.setdefault("AF_S4_SPLIT", "0")
import afpkg  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

from anchored_fusion_amd import _lib, discover, simworld  # noqa: E402
from anchored_fusion_amd import io as afio  # noqa: E402

N = int(os.environ.get("PAIRS", "50000000"))
L = 150
SCALE = float(os.environ.get("SCALE", "1.0"))
CAP = 400_000
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
dev = torch.device("cuda:0")
W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=SCALE)
ref = W.genome_index()
tiles = W.tiles()
reads_t = torch.empty((2 * N, L), dtype=torch.uint8, device=dev)
W.simulate_pairs(N, read_len=L, seed=20251015, pair_base=0, out=reads_t)
W.blob = None
torch.cuda.synchronize()
disc = discover.CandidateDiscovery(anchor, ref, tiles, N, L, device=0, inflight=4, batch_chunks=240, pair_base=0)
disc.run(reads_t)
torch.cuda.synchronize()
lib = _lib.lib()
lib.af_debug_g_prof_enable.argtypes = [ctypes.c_int64, ctypes.c_int32]
lib.af_debug_g_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int64]
GW = lib.af_debug_g_prof_enable(CAP, 4)
assert GW > 0
t0 = time.perf_counter()
disc.run(reads_t)
torch.cuda.synchronize()
print(f"profiled pass {time.perf_counter() - t0:.3f} s; {disc.summary()}")
buf = np.zeros((4, CAP, GW), dtype=np.int32)
ncalls = lib.af_debug_g_prof_read(buf.ctypes.data, buf.size)
if os.environ.get("GPROF_SAVE"):  # per-read interval counts and region counts of the first call
    np.save(os.environ["GPROF_SAVE"], buf[0][:, [1, 12, 13]].copy())
pct = lambda v, q: np.percentile(v, q) if len(v) else 0  # noqa: E731
for c in range(min(ncalls, 4)):
    B = buf[c]
    live = (B[:, 2] > 0) | (B[:, 0] != 0)
    n = int(live.sum())
    if not n:
        continue
    B = B[live].astype(np.int64)
    names = os.environ.get("GPROF_NAMES", "S4+S5 one launch").split(",")
    name = names[c] if c < len(names) else f"call {c}"
    print(f"== call {c}: {name}: {n} reads")
    g1 = B[:, 0] & 0xFFFFFFFF
    print(f"  G1 cycles/read mean {g1.mean():.0f} p50 {pct(g1, 50):.0f} p90 {pct(g1, 90):.0f} p99 {pct(g1, 99):.0f} "
          f"max {g1.max()}; intervals/read mean {B[:, 1].mean():.1f} max {B[:, 1].max()}")
    ext = B[:, 19] + B[:, 21] + B[:, 22]
    print(f"  G1 FM extensions/read mean {ext.mean():.0f} p50 {pct(ext, 50):.0f} p99 {pct(ext, 99):.0f} max {ext.max()}; "
          f"shares fwd {B[:, 19].sum() / max(ext.sum(), 1):.3f} bwd {B[:, 21].sum() / max(ext.sum(), 1):.3f} "
          f"seed-strategy {B[:, 22].sum() / max(ext.sum(), 1):.3f}; total {ext.sum()}")
    s1 = np.argsort(-g1)
    print("  G1 slowest: cycles wall_us | fwd bwd ss | len intervals")
    for i in s1[:8]:
        r = B[i]
        print(f"   {g1[i]:>11d} {((r[18] - r[17]) & 0xFFFFFFFF) / 100:8.1f} | {r[19]} {r[21]} {r[22]} | {r[2]} {r[1]}")
    cyc_per_ext = g1 / np.maximum(ext, 1)
    print(f"  G1 cycles per extension p50 {pct(cyc_per_ext, 50):.0f} p90 {pct(cyc_per_ext, 90):.0f}")
    if True:  # [23, 27) hold G1's trip split
        loop, extc, trips, iters = (B[:, 23].astype(np.int64) << 4, B[:, 24].astype(np.int64) << 4, B[:, 25], B[:, 26])
        ok = trips > 0
        print(f"  G1 per trip (wave time, S5 reads): bookkeeping loop {(loop[ok] / trips[ok]).mean():.0f} cycles, "
              f"FM extension {(extc[ok] / trips[ok]).mean():.0f} cycles, rest "
              f"{((g1[ok] - loop[ok] - extc[ok]) / trips[ok]).mean():.0f}; lane's loop iterations per trip "
              f"{(iters[ok] / trips[ok]).mean():.2f}")
    hw = B[:, 27] < 0  # G1's wave path (k_g_seeds_wave: -(cycles >> 4) - 1)
    n4 = 2 * int(disc.counts.get("s4_pairs", 0))  # the call's first 2 npair reads are S4's
    rid = np.nonzero(live)[0]
    for nm_, sel in (("S4", rid < n4), ("S5", rid >= n4)):
        h = hw & sel
        if h.any():
            wc_ = (-B[h, 27] - 1) << 4
            print(f"  G1 wave path, {nm_} reads: {int(h.sum())} of {int(sel.sum())}; cycles/read mean {wc_.mean():.0f} "
                  f"p99 {pct(wc_, 99):.0f} max {wc_.max()}; summed {wc_.sum() / 2.4e9 * 1e3:.1f} ms of one wave at 2.4 GHz")
    if hw.any():
        wc = (-B[hw, 27] - 1) << 4
        print(f"  G1 wave path: {int(hw.sum())} reads seen; cycles/read mean {wc.mean():.0f} p50 {pct(wc, 50):.0f} "
              f"max {wc.max()}; fwd steps mean {B[hw, 28].mean():.0f}, bwd positions mean {B[hw, 29].mean():.0f} "
              f"(entries {B[hw, 30].mean():.0f}), seed-strategy steps mean {B[hw, 31].mean():.0f}; "
              f"cycles per sequential step {(wc / np.maximum(B[hw, 28] + B[hw, 29] + B[hw, 31], 1)).mean():.0f}")
    lanes = B[:, 20]
    lane_sum = np.bincount(lanes, weights=g1)
    print(f"  G1 per-lane cycles: mean {lane_sum[lane_sum > 0].mean():.0f} max {lane_sum.max():.0f}")
    g2 = B[:, 3] & 0xFFFFFFFF
    ph = [B[:, k] & 0xFFFFFFFF for k in (4, 5, 6, 7)]
    print(f"  G2 cycles/read mean {g2.mean():.0f} p50 {pct(g2, 50):.0f} p90 {pct(g2, 90):.0f} p99 {pct(g2, 99):.0f} "
          f"p99.9 {pct(g2, 99.9):.0f} max {g2.max()}")
    tot = max(g2.sum(), 1)
    print("  G2 shares: " + ", ".join(f"{nm} {v.sum() / tot:.3f}" for nm, v in zip(("chain", "flt", "ext", "dedup"), ph)))
    srt = np.argsort(-g2)
    top = g2[srt[:100]].sum() / tot
    print(f"  top-100 reads hold {top:.3f} of G2 cycles; top-1000 {g2[srt[:1000]].sum() / tot:.3f}")
    print("  heaviest: cyc chain flt (its sort) ext dedup | len niv occ nch kept nreg nreg2")
    for i in srt[:12]:
        r = B[i]
        print(f"   {g2[i]:>11d} {ph[0][i]:>10d} {ph[1][i]:>9d} ({r[43]:>8d}) {ph[2][i]:>10d} {ph[3][i]:>9d} | {r[2]} {r[1]} "
              f"{r[8]} {r[10]} {r[11]} {r[12]} {r[13]}")
    for k, nm in ((8, "occ"), (10, "chains"), (11, "kept"), (12, "regions")):
        v = B[:, k]
        print(f"  {nm:8s} mean {v.mean():.1f} p90 {pct(v, 90):.0f} p99 {pct(v, 99):.0f} max {v.max()}")
    # schedule (s_memrealtime, 100 MHz, the low 32 bits: times as signed offsets from one stamp,
    # wrap-safe; rows a kernel did not stamp left out)
    def rel(t0, t1):
        ok = (t0 != 0) | (t1 != 0)
        base = int(t0[ok][0]) if ok.any() else 0
        d0 = ((t0 - base + (1 << 31)) % (1 << 32)) - (1 << 31)
        d1 = ((t1 - base + (1 << 31)) % (1 << 32)) - (1 << 31)
        return ok, d0, d1
    ok2, t0_, t1_ = rel(B[:, 15] & 0xFFFFFFFF, B[:, 16] & 0xFFFFFFFF)
    if ok2.any():
        lo = t0_[ok2].min()
        busy = np.bincount(B[ok2, 14], weights=(t1_[ok2] - t0_[ok2]))
        print(f"  G2 makespan {(t1_[ok2].max() - lo) / 100:.0f} us; per-wave busy mean {busy[busy > 0].mean() / 100:.0f} us "
              f"max {busy.max() / 100:.0f} us over {int((busy > 0).sum())} waves; last read starts at "
              f"{(t0_[ok2].max() - lo) / 100:.0f} us")
    ok1, tg0, tg1 = rel(B[:, 17] & 0xFFFFFFFF, B[:, 18] & 0xFFFFFFFF)
    if ok1.any():
        w1 = tg1[ok1] - tg0[ok1]
        print(f"  G1 (lane path) makespan {(tg1[ok1].max() - tg0[ok1].min()) / 100:.0f} us over {int(ok1.sum())} reads; "
              f"per-read wall p50 {pct(w1, 50) / 100:.1f} us p99 {pct(w1, 99) / 100:.1f} us max {w1.max() / 100:.1f} us")
    # k_g_heavy (fields [40, 43): its start / end stamps and wave): the reads G2 deferred
    H = B[(B[:, 40] != 0) | (B[:, 41] != 0)]
    if len(H):
        hc = (H[:, 6] & 0xFFFFFFFF) + (H[:, 7] & 0xFFFFFFFF)
        okh, t0_, t1_ = rel(H[:, 40] & 0xFFFFFFFF, H[:, 41] & 0xFFFFFFFF)
        lo = t0_[okh].min()
        busy = np.bincount(H[okh, 42], weights=(t1_[okh] - t0_[okh]))
        print(f"  heavy reads (k_g_heavy) {len(H)}: cycles/read mean {hc.mean():.0f} p99 {pct(hc, 99):.0f} max {hc.max()}; "
              f"summed {hc.sum() / 2.4e9 * 1e3:.1f} ms of one wave at 2.4 GHz; makespan {(t1_[okh].max() - lo) / 100:.0f} us "
              f"over {int((busy > 0).sum())} waves (busy mean {busy[busy > 0].mean() / 100:.0f} us max {busy.max() / 100:.0f} us); "
              f"last read starts at {(t0_[okh].max() - lo) / 100:.0f} us; per-read wall max {(t1_[okh] - t0_[okh]).max() / 100:.0f} us")
    # k_g_pe (rows of the pairs' first reads, fields [32, 40)): rescue (ksw_align2 + dedup), pairing, records
    P = B[(B[:, 38] != 0) | (B[:, 39] != 0)]
    if len(P):
        resc, pair, rec = P[:, 32], P[:, 33], P[:, 34]
        tot = resc + pair + rec
        print(f"  PE {len(P)} pairs: cycles/pair mean {tot.mean():.0f} p50 {pct(tot, 50):.0f} p99 {pct(tot, 99):.0f} "
              f"max {tot.max()}; shares rescue {resc.sum() / tot.sum():.3f} (dedup {P[:, 36].sum() / tot.sum():.3f}) "
              f"pair {pair.sum() / tot.sum():.3f} records {rec.sum() / tot.sum():.3f}")
        print(f"  PE ksw_align2 calls/pair mean {P[:, 35].mean():.2f} p99 {pct(P[:, 35], 99):.0f} max {P[:, 35].max()}; "
              f"pairs with >= 8: {(P[:, 35] >= 8).sum()} holding {resc[P[:, 35] >= 8].sum() / tot.sum():.3f} of the cycles")
        sp = np.argsort(-tot)
        print(f"  PE top-100 pairs hold {tot[sp[:100]].sum() / tot.sum():.3f}; top-1000 {tot[sp[:1000]].sum() / tot.sum():.3f}")
        print("  PE heaviest: cyc rescue dedup pair records | ksw na0 na1")
        for i in sp[:12]:
            r = P[i]
            print(f"   {tot[i]:>11d} {r[32]:>10d} {r[36]:>10d} {r[33]:>9d} {r[34]:>9d} | {r[35]} {r[37] >> 16} {r[37] & 0xFFFF}")
        okp, t0_, t1_ = rel(P[:, 38] & 0xFFFFFFFF, P[:, 39] & 0xFFFFFFFF)
        lo = t0_[okp].min()
        print(f"  PE makespan {(t1_[okp].max() - lo) / 100:.0f} us; last pair starts at {(t0_[okp].max() - lo) / 100:.0f} us; "
              f"per-pair wall p50 {pct(t1_[okp] - t0_[okp], 50) / 100:.1f} us max {(t1_[okp] - t0_[okp]).max() / 100:.1f} us")
disc.close()
