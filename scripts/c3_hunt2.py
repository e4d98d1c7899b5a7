"""Debug aid: align chosen pairs of the dumped sample on the GPU, compare with the oracle."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: F401
import numpy as np
import oracle
from anchored_fusion_amd import io as afio
from anchored_fusion_amd.align import AnchorAligner
d = np.load(sys.argv[1])
reads = d["reads"]
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
al = AnchorAligner(anchor, device=0)
ix = oracle.OracleIndex(anchor)
for spec in sys.argv[2:]:
    if ":" in spec:
        a, b = map(int, spec.split(":"))
        pairs = np.arange(a, b)
    else:
        pairs = np.array([int(v) for v in spec.split(",")])
    rows = np.stack([2 * pairs, 2 * pairs + 1], 1).reshape(-1)
    sub = reads[rows]
    print(f"{spec}: {len(pairs)} pairs ...", flush=True)
    t0 = time.time()
    r = al.align_pairs(sub)
    o = ix.align_pairs(sub)
    same = all(np.array_equal(getattr(r, k), o[k]) for k in ("flag", "pos", "score", "n_cigar"))
    print(f"{spec}: {time.time() - t0:.2f} s, mapped {int(r.mapped().sum())}, equal to oracle {same}", flush=True)
