"""Per-candidate phase cycles of the lane-per-read K2 (profiling build; AF_GPU_LIB=libafgpu_prof.so)."""
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
lib.af_debug_lane_prof_enable.argtypes = [ctypes.c_int64]
lib.af_debug_lane_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int64]
assert lib.af_debug_lane_prof_enable(nr) == 8
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
buf = np.zeros((nc, 8), dtype=np.int32)
assert lib.af_debug_lane_prof_read(buf.ctypes.data, nc) == 0
for k, nm in ((1, "load"), (2, "mem"), (3, "ext"), (4, "cigar"), (5, "trace")):
    v = buf[:, k].astype(np.int64)
    print(f"  {nm:6s} mean {v.mean():.0f}  p50 {np.median(v):.0f}  p90 {np.percentile(v, 90):.0f}  max {v.max()}")
