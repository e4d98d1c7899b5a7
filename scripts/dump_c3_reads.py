"""Dump a small configs[2]-style read sample made on the device (debug aid: the reads can then be
aligned by the CPU oracle here)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: F401
import numpy as np
import torch
from anchored_fusion_amd import io as afio, simworld
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=float(sys.argv[1]))
n = int(sys.argv[2])
src = torch.zeros(n, dtype=torch.int32, device="cuda:0")
r = W.simulate_pairs(n, read_len=150, seed=20251015, src=src)
torch.cuda.synchronize()
os.makedirs(sys.argv[3], exist_ok=True)
np.savez_compressed(os.path.join(sys.argv[3], "reads.npz"), reads=r.cpu().numpy(), src=src.cpu().numpy(),
                    junctions=np.array(W.junctions), fusions=np.array([f.decode() for f in W.fusions]))
print("dumped", n)
