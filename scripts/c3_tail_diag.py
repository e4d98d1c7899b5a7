"""Debug aid: which split-read tails of the configs[2] world place outside the embedded genes."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: F401
import numpy as np
import torch
from anchored_fusion_amd import discover, simworld
from anchored_fusion_amd import io as afio
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
scale, N = float(sys.argv[1]), int(sys.argv[2])
W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=scale)
ref = W.reference()
src = torch.zeros(N, dtype=torch.int32, device="cuda:0")
reads_t = W.simulate_pairs(N, read_len=150, seed=20251015, src=src)
d = discover.CandidateDiscovery(anchor, ref, N, 150, device=0)
d.run(reads_t)
rows, nh, best = d.tail_best_hits()
spans = [(W.names.index(v[0][0]), v[0][1] - 1000, v[-1][2] + 1000, k) for k, v in W.loci.items()]
out = []
srcs = src.cpu().numpy()
tl = d.tails["lens"].cpu().numpy()
tq = d.tails["tails"].cpu().numpy()
flag = d.out["flag"].cpu().numpy(); pos = d.out["pos"].cpu().numpy()
for t in np.nonzero(nh > 0)[0]:
    loc = ref.locate(best[t]["t_start"], best[t]["t_end"])
    hit = None if loc is None else next((k for c, s, e, k in spans if c == loc[0] and s <= loc[1] < e), None)
    if hit is None and len(out) < 300:
        r = int(rows[t])
        out.append(dict(row=r, src=int(srcs[r // 2]), flag=int(flag[r]), pos=int(pos[r]), tail=tq[t, :tl[t]].tobytes().decode(),
                        n_hits=int(nh[t]), score=int(best[t]["score"]), ctg=None if loc is None else W.names[loc[0]],
                        at=None if loc is None else int(loc[1]), read=reads_t[r].cpu().numpy().tobytes().decode()))
json.dump(dict(loci={k: v for k, v in W.loci.items()}, junctions=W.junctions, bad=out), open(sys.argv[3], "w"), indent=1)
print("dumped", len(out))
