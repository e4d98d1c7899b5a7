"""Debug aid: align the dumped configs[2] sample (scripts/dump_c3_reads.py) chunk by chunk on the GPU
and compare with the CPU oracle records written by the same script's caller."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: F401
import numpy as np
from anchored_fusion_amd import io as afio
from anchored_fusion_amd.align import AnchorAligner
d = np.load(sys.argv[1])
reads = d["reads"]
step = int(sys.argv[2])
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
al = AnchorAligner(anchor, device=0)
for lo in range(0, reads.shape[0] // 2, step):
    t0 = time.time()
    print(f"chunk {lo} ...", flush=True)
    r = al.align_pairs(reads[2 * lo:2 * (lo + step)])
    print(f"chunk {lo}: {time.time() - t0:.2f} s, mapped {int(r.mapped().sum())}", flush=True)
