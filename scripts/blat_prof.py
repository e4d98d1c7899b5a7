"""Per-query phase cycles of k_blat on the configs[2] S6 queries (the QNAME-group leaders searched
beside S5, `s6p`; profiling build libafgpu_prof.so; one strand's row per query: the strands of a
query share it, the last written wins), split into the queries S5's check keeps and drops.

python scripts/blat_prof.py [pairs] [out.json]   (GPU; make -C anchored-fusion_amd/csrc prof first)
"""
import json
import os
import sys

os.environ["AF_GPU_LIB"] = "libafgpu_prof.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: F401,E402
import numpy as np  # noqa: E402
import torch  # noqa: E402

from anchored_fusion_amd import _lib, discover, simworld  # noqa: E402
from anchored_fusion_amd import io as afio  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/blat_prof.json"
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=1.0)
ref, tiles = W.genome_index(), W.tiles()
reads = W.simulate_pairs(N, read_len=150, seed=20251015)
L = _lib.lib()
assert L.af_debug_blat_prof_enable() == 16
W.blob = None
d = discover.CandidateDiscovery(anchor, ref, tiles, N, 150, device=0, inflight=4, batch_chunks=240)
d.run(reads)
torch.cuda.synchronize()
nt = min(int(d.s6p["n"].item()), d.s6cap)
n6 = int(d.s6["n"].item())
pre_src = d.s6p["src"][:nt].cpu().numpy()
kept = np.isin(pre_src, d.s6["src"][:n6].cpu().numpy())
P = np.zeros((nt, 16), dtype=np.int32)
assert L.af_debug_blat_prof_read(P.ctypes.data_as(__import__("ctypes").c_void_p), nt) == 0
names = ["hits", "sort", "clumps", "hsp", "chain"]
tot = P[:, 9].astype(np.int64)
res = dict(queries=nt, mean_cycles={n: float(P[:, k].mean()) for k, n in enumerate(names)},
           mean_total=float(tot.mean()), mean_filter_cycles=float(P[:, 10].mean()), mean_kept=float(P[:, 11].mean()), pct_total={p: float(np.percentile(tot, p)) for p in (50, 90, 99, 99.9)},
           mean_hits=float(P[:, 5].mean()), mean_clumps=float(P[:, 6].mean()), mean_parts=float(P[:, 7].mean()),
           mean_ranges=float(P[:, 13].mean()), mean_deferred=float(P[:, 12].mean()),
           mean_len=float(P[:, 8].mean()),
           kept=int(kept.sum()), dropped=int((~kept).sum()),
           cycles_kept=int(tot[kept].sum()), cycles_dropped=int(tot[~kept].sum()),
           max_kept=int(tot[kept].max()) if kept.any() else 0, max_dropped=int(tot[~kept].max()) if (~kept).any() else 0,
           slowest=[dict(zip(names + ["hits_n", "clumps_n", "parts_n", "len", "total"], map(int, P[i, :10])),
                         kept=bool(kept[i])) for i in np.argsort(-tot)[:40]])
# share of the summed cycles in the slowest 1% of the queries
o = np.sort(tot)[::-1]
res["top1pct_share"] = float(o[:max(1, nt // 100)].sum() / max(1, o.sum()))
os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "slowest"}, indent=1))
