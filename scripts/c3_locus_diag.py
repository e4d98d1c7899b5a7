"""Debug aid: print genome windows of the configs[2] world."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: F401
import numpy as np
from anchored_fusion_amd import simworld
from anchored_fusion_amd import io as afio
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=1.0)
print("partner2 locus", W.loci["partner2"][:3])
for spec in sys.argv[1:]:
    c, p = spec.split(":")
    o = W.offsets[W.names.index(c)] + int(p)
    print(spec, W.blob[o - 20:o + 140].cpu().numpy().tobytes().decode())
# count occurrences of a partner-2 25-mer in the whole genome (chunked)
t = np.frombuffer(b"TCGTTTGCTTCTCGCGCCGTCTTGG", np.uint8)
import torch
tt = torch.from_numpy(t.copy()).cuda()
hits = []
B = 1 << 28
for s in range(0, W.total - 25, B):
    blk = W.blob[s:min(W.total, s + B + 24)]
    m = blk[:-24] == tt[0]
    for k in range(1, 25):
        m &= blk[k:k + len(blk) - 24] == tt[k]
    idx = torch.nonzero(m).flatten().cpu().numpy() + s
    hits += idx.tolist()
print("occurrences", len(hits), [(W.names[np.searchsorted(W.offsets, h, side='right') - 1], h - W.offsets[np.searchsorted(W.offsets, h, side='right') - 1]) for h in hits[:10]])
