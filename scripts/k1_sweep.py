"""K1 scaling probe: time vs batch size, against torch copy/sum on the same buffer."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

from anchored_fusion_amd import io as afio  # noqa: E402
from anchored_fusion_amd import simulate as sim  # noqa: E402
from anchored_fusion_amd.align import AnchorAligner  # noqa: E402

anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
_, base, _, _ = sim.fusion_reads(anchor, 1_000_000, read_len=100, fusion_frac=0.05, seed=20251015)
dev = torch.device("cuda:0")
al = AnchorAligner(anchor)
s = torch.cuda.current_stream()


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for mult in (0.25, 1, 4):
    n = int(1_000_000 * mult)
    reads = np.tile(base, (int(np.ceil(mult)), 1))[: 2 * n]
    rt = torch.from_numpy(np.ascontiguousarray(reads)).to(dev)
    hits = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    us = timeit(lambda: al.seed_filter_device(rt, 2 * n, 100, hits, stream=s))
    out = torch.empty_like(rt)
    cp = timeit(lambda: out.copy_(rt))
    rt32 = rt.view(torch.int32)
    sm = timeit(lambda: rt32.sum())
    print(f"pairs={n:>8} k1={us:8.1f}us ({rt.numel() / us / 1e3:7.1f} GB/s)  copy={cp:7.1f}us "
          f"({2 * rt.numel() / cp / 1e3:7.1f} GB/s)  sum={sm:7.1f}us ({rt.numel() / sm / 1e3:7.1f} GB/s)", flush=True)
