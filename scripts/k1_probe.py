"""Runs only the seed filter (K1) on the bench workload, for rocprofv3 counter passes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: E402,F401
import torch  # noqa: E402

from anchored_fusion_amd import io as afio  # noqa: E402
from anchored_fusion_amd import simulate as sim  # noqa: E402
from anchored_fusion_amd.align import AnchorAligner  # noqa: E402

n = int(os.environ.get("PAIRS", "1000000"))
iters = int(os.environ.get("ITERS", "10"))
L = int(os.environ.get("READ_LEN", "100"))
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
_, reads, _, _ = sim.fusion_reads(anchor, n, read_len=L, fusion_frac=0.05, seed=20251015)
dev = torch.device("cuda:0")
rt = torch.from_numpy(reads).to(dev)
hits = torch.zeros(reads.shape[0], dtype=torch.int32, device=dev)
al = AnchorAligner(anchor)
s = torch.cuda.current_stream()
for _ in range(2):
    al.seed_filter_device(rt, reads.shape[0], L, hits, stream=s)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(iters):
    al.seed_filter_device(rt, reads.shape[0], L, hits, stream=s)
e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
print(f"k1 {ms * 1e3:.1f} us/launch  {reads.nbytes / (ms * 1e-3) / 1e9:.1f} GB/s  cand={al.last_candidates()}")
# the bench's way: events around each launch (the step's other kernels absent)
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(iters)]
for k in range(iters):
    evs[k][0].record(s)
    al.seed_filter_device(rt, reads.shape[0], L, hits, stream=s)
    evs[k][1].record(s)
torch.cuda.synchronize()
ms1 = sum(a.elapsed_time(b) for a, b in evs) / iters
print(f"k1 per-launch events {ms1 * 1e3:.1f} us/launch")
