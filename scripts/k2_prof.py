"""K2 per-candidate phase profile (profiling build libafgpu_prof.so; run with AF_GPU_LIB=libafgpu_prof.so).

Prints the distribution of per-read cycles by phase (MEM search, seed extension, CIGAR) and the
per-slot load balance; saves the raw table to gpurun_out/k2prof.npy.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("AF_GPU_LIB", "libafgpu_prof.so")
import afpkg  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

from anchored_fusion_amd import _lib  # noqa: E402
from anchored_fusion_amd import io as afio  # noqa: E402
from anchored_fusion_amd import simulate as sim  # noqa: E402
from anchored_fusion_amd.align import AnchorAligner  # noqa: E402

n = int(os.environ.get("PAIRS", "1000000"))
L = int(os.environ.get("READ_LEN", "100"))
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
_, reads, _, _ = sim.fusion_reads(anchor, n, read_len=L, fusion_frac=0.05, seed=20251015)
dev = torch.device("cuda:0")
rt = torch.from_numpy(reads).to(dev)
nr = reads.shape[0]
out = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
out["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
lib = _lib.lib()
lib.af_debug_k2_prof_enable.argtypes = [ctypes.c_int64]
lib.af_debug_k2_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int64]
W = lib.af_debug_k2_prof_enable(nr)
assert W > 0
al = AnchorAligner(anchor)
s = torch.cuda.current_stream()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
for it in range(3):
    e[0].record(s)
    al.seed_filter_device(rt, nr, L, out["hits"], stream=s)
    e[1].record(s)
    al.align_candidates_device(rt, n, L, out, stream=s)
    e[2].record(s)
    torch.cuda.synchronize()
    print(f"iter {it}: k1 {e[0].elapsed_time(e[1]) * 1e3:.1f} us  k2+k3 {e[1].elapsed_time(e[2]) * 1e3:.1f} us")
nc = al.last_candidates()
buf = np.zeros((nc, W), dtype=np.int32)
assert lib.af_debug_k2_prof_read(buf.ctypes.data, nc) == 0
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", "k2prof.npy"), buf)
names = ["read", "total", "mem", "ext", "cigar", "nmem", "nreg", "ext_rows", "cig_rows", "ext_dp", "ext_calls", "traceback"]
T = buf[:, 1].astype(np.int64)
print(f"candidates {nc}; cycles/read mean {T.mean():.0f} p50 {np.median(T):.0f} p90 {np.percentile(T, 90):.0f} "
      f"p99 {np.percentile(T, 99):.0f} max {T.max()}")
for k, nm in ((2, "mem"), (3, "ext"), (9, "ext_dp"), (4, "cigar"), (11, "trace")):
    v = buf[:, k].astype(np.int64)
    print(f"  {nm:6s} share {v.sum() / T.sum():.3f}  mean {v.mean():.0f}  p99 {np.percentile(v, 99):.0f}")
for k in (5, 6, 7, 8, 10):
    v = buf[:, k]
    print(f"  {names[k]:9s} mean {v.mean():.2f} p90 {np.percentile(v, 90):.0f} max {v.max()}")
mapped = buf[:, 6] > 0
print(f"  reads with regions {mapped.sum()}  cycles/read with regions {T[mapped].mean():.0f}, "
      f"without {T[~mapped].mean() if (~mapped).any() else 0:.0f}")
for nm, (cc, rr) in (("ext w1", (12, 13)), ("ext gen", (14, 15))):
    c, r = buf[:, cc].astype(np.int64).sum(), buf[:, rr].astype(np.int64).sum()
    print(f"  {nm}: rows {r} cycles/row {c / max(r, 1):.0f} share of ext_dp {c / max(buf[:, 9].astype(np.int64).sum(), 1):.3f}")
# cycles per extension row and per cigar row (least squares over reads with work)
A = np.stack([buf[:, 7], buf[:, 8], np.ones(nc)], 1).astype(np.float64)
coef, *_ = np.linalg.lstsq(A, (buf[:, 3] + buf[:, 4]).astype(np.float64), rcond=None)
print(f"  fit ext+cigar cycles ~ {coef[0]:.0f}*ext_rows + {coef[1]:.0f}*cig_rows + {coef[2]:.0f}")
if W >= 19:
    # schedule: per-slot busy spans from s_memrealtime (100 MHz), the makespan and its tail
    slot, t0, t1 = buf[:, 16], buf[:, 17].astype(np.int64), buf[:, 18].astype(np.int64)
    base = t0.min()
    t0, t1 = (t0 - base) & 0xFFFFFFFF, (t1 - base) & 0xFFFFFFFF
    span = t1.max()
    last = np.zeros(slot.max() + 1, np.int64)
    np.maximum.at(last, slot, t1)
    busy = np.zeros(slot.max() + 1, np.int64)
    np.add.at(busy, slot, t1 - t0)
    q = np.percentile(last, [1, 50, 99])
    print(f"  schedule: makespan {span / 100:.1f} us; slot finish p1 {q[0] / 100:.1f} p50 {q[1] / 100:.1f} "
          f"p99 {q[2] / 100:.1f} us; mean slot busy {busy.mean() / 100:.1f} us; "
          f"items started after 90% of the makespan {(t0 > 0.9 * span).sum()}; longest item {(t1 - t0).max() / 100:.1f} us")
    late = np.argsort(t1)[-5:]
    for k in late:
        print(f"    late item {k}: start {t0[k] / 100:.1f} end {t1[k] / 100:.1f} us, hits {int(out['hits'][int(buf[k, 0])])}, "
              f"nmem {buf[k, 5]} nreg {buf[k, 6]} ext_rows {buf[k, 7]} cig_rows {buf[k, 8]}")
