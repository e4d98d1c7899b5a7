"""Times the homolog search (fn:341: the anchor transcript as one BLAT query against the genome,
preset "homologs": step 3, repMatch 10000) on the configs[2] world: the step-3 tile index build
and af_blat_long, separately.  Run under rocprofv3 --kernel-trace --stats for the per-kernel split.

    python scripts/homolog_prof.py [scale]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: E402,F401
import torch  # noqa: E402

from anchored_fusion_amd import blat  # noqa: E402
from anchored_fusion_amd import io as afio  # noqa: E402
from anchored_fusion_amd import simworld  # noqa: E402

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=scale)
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    T = W.tiles(step_size=3)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    rows, n, blocks, boff = T.search_long(anchor, blat.params("homologs"))
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"pass {rep}: step-3 tile index {t1 - t0:.2f} s, af_blat_long {t2 - t1:.2f} s, rows {int(n)}", flush=True)
    T.close()
