"""Debug: G1 intervals vs the oracle's on a few reads of the test genome world."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import afpkg  # noqa: F401,E402
import numpy as np  # noqa: E402
import oracle  # noqa: E402
from genome_world import make_genome, sample_reads  # noqa: E402
from anchored_fusion_amd.genome import GenomeIndex  # noqa: E402
contigs = make_genome()
og, gg = oracle.OracleGenome(contigs), GenomeIndex(contigs, device=0)
reads, lens = sample_reads(contigs, 6, seed=20, chimeric=0.4)
io, no = og.intervals(reads, lens, threads=1)
ig, ng = gg.intervals(reads, lens)
for r in range(6):
    print("read", r, "len", lens[r], "oracle", no[r], "gpu", ng[r])
    print("  oracle:", [tuple(int(v) for v in io[r, k]) for k in range(no[r])])
    print("  gpu:   ", [tuple(int(v) for v in ig[r, k]) for k in range(ng[r])])
