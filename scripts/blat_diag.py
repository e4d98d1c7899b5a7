"""Debug aid: time the BLAT search of configs[2] split-read tails by group."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: F401
import numpy as np
import torch
from anchored_fusion_amd import blat, discover, simworld
from anchored_fusion_amd import io as afio
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=1.0)
ref = W.reference(); tiles = W.tiles()
N = 5_000_000
reads_t = W.simulate_pairs(N, read_len=150, seed=20251015)
d = discover.CandidateDiscovery(anchor, ref, tiles, N, 150, device=0)
d.run(reads_t)
torch.cuda.synchronize()
nt = int(d.tails["n"].item())
tl = d.tails["lens"][:nt].cpu().numpy()
tq = d.tails["tails"][:nt].cpu().numpy()
seqs = [tq[i, :tl[i]].tobytes().decode() for i in range(nt)]
p = blat.params("split_tail")
t0 = time.time(); rows, nr = tiles.search(seqs, p); dt = time.time() - t0
print(f"{nt} tails: {dt*1e3:.1f} ms host-API; rows/tail {np.bincount(nr)}", flush=True)
lens = np.array([len(s) for s in seqs])
for lo, hi in ((0, 40), (40, 80), (80, 200)):
    sel = [s for s in seqs if lo <= len(s) < hi][:2000]
    t0 = time.time(); tiles.search(sel, p); dt = time.time() - t0
    print(f"len [{lo},{hi}): {len(sel)} tails {dt*1e3:.1f} ms", flush=True)
# per-tail cost: time tails one at a time for a sample
costs = []
for i in range(0, nt, max(1, nt // 200)):
    t0 = time.time(); tiles.search([seqs[i]], p); costs.append((time.time() - t0, i))
costs.sort(reverse=True)
for c, i in costs[:8]:
    print(f"  {c*1e3:.2f} ms len {len(seqs[i])} rows {nr[i]} {seqs[i][:60]}")
print("median single", sorted(c for c, _ in costs)[len(costs)//2]*1e3, "ms")
