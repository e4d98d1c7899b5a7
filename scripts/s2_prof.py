"""S2 per-item phase profile (profiling build libafgpu_prof.so, `make -C anchored-fusion_amd/csrc prof`).

K2 (k_s2_regions) per candidate read: seeding (MEMs + SMEM passes), chaining (lane 0),
extension, dedup/patch.  K3c (k_s2_pairs) per listed pair: load, mate rescue, primary/pairing,
records (CIGAR).  Prints mean cycles per phase and the counts behind them.
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
dev = torch.device("cuda:0")
if os.environ.get("WORLD") == "c3":  # the configs[2] world (simworld): reads from the genome + fusions
    from anchored_fusion_amd import simworld
    W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=1.0)
    rt = W.simulate_pairs(n, read_len=L, seed=20251015)
    del W
else:
    _, reads, _, _ = sim.fusion_reads(anchor, n, read_len=L, fusion_frac=0.05, seed=20251015)
    rt = torch.from_numpy(reads).to(dev)
nr = rt.shape[0]
out = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
out["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
lib = _lib.lib()
lib.af_debug_s2_prof_enable.argtypes = []
lib.af_debug_s2_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
assert lib.af_debug_s2_prof_enable() > 0
al = AnchorAligner(anchor)
for it in range(2):
    al.align_pairs_device(rt, nr // 2, L, out)
    torch.cuda.synchronize()
h = out["hits"].cpu().numpy()
n_k2 = int((h > 0).sum())
n_k3 = int((((h[0::2] > 0) | (h[1::2] > 0))).sum())
buf = np.zeros(16 * (n_k2 + n_k3), dtype=np.int32)
assert lib.af_debug_s2_prof_read(buf.ctypes.data, n_k2, n_k3) == 0
k2 = buf[:16 * n_k2].reshape(-1, 16).astype(np.int64)
k3 = buf[16 * n_k2:].reshape(-1, 16).astype(np.int64)
print(f"K2: {n_k2} reads; mean cycles total {k2[:, 1].mean():.0f}: seed {k2[:, 2].mean():.0f}, chain "
      f"{k2[:, 3].mean():.0f}, extend {k2[:, 4].mean():.0f}, dedup {k2[:, 5].mean():.0f}")
sub = k2[:, 6] >> 8
k2[:, 6] &= 0xFF
print(f"    seeding: read load {k2[:, 12].mean():.0f}, MEMs {k2[:, 13].mean():.0f}, pass 1 {k2[:, 14].mean():.0f}, "
      f"pass 2 {k2[:, 15].mean():.0f}, pass 3 {sub.mean():.0f}")
rows, calls = k2[:, 11] >> 8, k2[:, 11] & 0xFF
print(f"    extension: ksw_extend2 calls/read {calls.mean():.2f}, rows/read {rows.mean():.1f}, rows/call "
      f"{rows.sum() / max(calls.sum(), 1):.1f}, cycles/row {k2[:, 4].sum() / max(rows.sum(), 1):.0f}; reads with no "
      f"extension {(calls == 0).mean():.3f}")
print(f"    MEMs {k2[:, 6].mean():.2f}, intervals {k2[:, 7].mean():.2f}, chains {k2[:, 8].mean():.2f}, "
      f"regions {k2[:, 9].mean():.2f} -> {k2[:, 10].mean():.2f}")
resc = k3[:, 6] > 0
print(f"K3c: {n_k3} pairs; mean cycles total {k3[:, 1].mean():.0f}: load {k3[:, 2].mean():.0f}, rescue "
      f"{k3[:, 3].mean():.0f}, primary/pair {k3[:, 4].mean():.0f}, records {k3[:, 5].mean():.0f}")
print(f"    pairs with a rescue SW {resc.sum()} (window rows {k3[resc, 6].mean() if resc.any() else 0:.0f}); "
      f"their rescue cycles {k3[resc, 3].mean() if resc.any() else 0:.0f}, others {k3[~resc, 3].mean():.0f}")
for q in (50, 90, 99):
    print(f"    p{q}: K2 total {np.percentile(k2[:, 1], q):.0f}, K3c total {np.percentile(k3[:, 1], q):.0f}")
top = np.argsort(-k3[:, 1])[:12]
print("K3c slowest pairs: pair, total, load, rescue, primary, records, rescue rows, regions m1/m2")
for t in top:
    print("   ", k3[t, [0, 1, 2, 3, 4, 5, 6, 7, 8]].tolist())
print(f"K3c cycles: sum {k3[:, 1].sum():.3g}, of which rescue {k3[:, 3].sum():.3g}; max {k3[:, 1].max()}")
