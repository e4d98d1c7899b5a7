"""Genome-scale placement (SURVEY.md §8 f rank 2, configs C3/C4's HBM-resident genome index):
builds af_index_build_genome over a random genome of G bases (default 3.1 G, 24 contigs), then
places Q reads of 150 bp drawn from it (half reverse-complemented) with af_place and checks the
best hit of each against its source.

usage: python3 scripts/genome_bench.py [G] [Q]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: E402,F401
import numpy as np  # noqa: E402

from anchored_fusion_amd import place  # noqa: E402

G = int(float(sys.argv[1])) if len(sys.argv) > 1 else 3_100_000_000
Q = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
rng = np.random.default_rng(20251015)
n_ctg = 24
acgt = np.frombuffer(b"ACGT", np.uint8)
t0 = time.perf_counter()
ctgs = []
for k in range(n_ctg):
    a = acgt[rng.integers(0, 4, G // n_ctg, dtype=np.uint8)]
    ctgs.append((f"chr{k + 1}", a.tobytes().decode()))
    print(f"contig {k + 1}/{n_ctg} generated ({time.perf_counter() - t0:.0f} s)", flush=True)
t1 = time.perf_counter()
ref = place.Reference(ctgs)
t2 = time.perf_counter()
print(f"index ({ref.kind}) of {ref.total / 1e9:.2f} Gbp built in {t2 - t1:.2f} s (incl. host join + H2D)",
      flush=True)
comp = str.maketrans("ACGT", "TGCA")
seqs, truth = [], []
for i in range(Q):
    k = int(rng.integers(n_ctg))
    s = int(rng.integers(0, len(ctgs[k][1]) - 150))
    q = ctgs[k][1][s:s + 150]
    rev = bool(i & 1)
    seqs.append(q.translate(comp)[::-1] if rev else q)
    truth.append((k, s, rev))
p = place._lib.default_params()
ref.raw_hits(seqs[:1000], p, 4)
t3 = time.perf_counter()
g, gn = ref.raw_hits(seqs, p, 4)
t4 = time.perf_counter()
ok = 0
for i, (k, s, rev) in enumerate(truth):
    if gn[i] >= 1:
        loc = ref.locate(g[i, 0]["t_start"], g[i, 0]["t_end"])
        ok += loc is not None and loc[0] == k and loc[1] == s and bool(g[i, 0]["flag"] & 0x10) == rev
print(f"placed {Q} x 150 bp reads in {t4 - t3:.3f} s = {Q / (t4 - t3) / 1e6:.2f} M reads/s "
      f"(host API incl. H2D/D2H); best hit at the source for {ok}/{Q}", flush=True)
ref.close()
