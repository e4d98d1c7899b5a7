"""Single-cell leg (configs[4] scaled to one GPU): C cells x P pairs of 2x100 through
`singlecell.run` -- cells batched into GPU alignment passes, S3-S8 per cell, the SC:258-287
merge.  Each cell holds a slice of tests/fusion_world.make_world's fusion/anchor pairs plus
vectorised background fragments of the world genome, written as a BGZF FASTQ pair.  Prints one
JSON line (cells/s, pairs/s, the merged fusion row).

    python scripts/sc_bench.py [cells] [pairs_per_cell] [out.json]
"""
import json
import os
import sys
import time
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import afpkg  # noqa: E402,F401
import numpy as np  # noqa: E402
from e2e_bench import fastq_bytes, write_bgzf  # noqa: E402


def main():
    n_cells = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    out = sys.argv[3] if len(sys.argv) > 3 else None
    from fusion_world import make_world
    from anchored_fusion_amd import io as afio
    from anchored_fusion_amd import singlecell
    folder = os.path.join(os.environ.get("TMPDIR", "/tmp"), "af_sc")
    cells_dir = os.path.join(folder, "cells")
    os.makedirs(cells_dir, exist_ok=True)
    t0 = time.perf_counter()
    paths, truth = make_world(folder, n_fusion=4000, n_anchor=3000, n_background=100)
    genome = np.concatenate([np.frombuffer(s, dtype=np.uint8) for _, s in afio.read_fasta(paths["genome"])])
    _, reads0, _ = afio.read_pairs(paths["fq1"], paths["fq2"])
    L = reads0.shape[1]
    k0 = reads0.shape[0] // 2
    rng = np.random.default_rng(11)
    comp = np.zeros(256, dtype=np.uint8)
    for a, b in zip(b"ACGTN", b"TGCAN"):
        comp[a] = b
    with Pool(min(16, os.cpu_count() or 1)) as pool:
        for c in range(n_cells):
            lo, hi = c * k0 // n_cells, (c + 1) * k0 // n_cells  # this cell's fusion / anchor pairs
            m = per - (hi - lo)
            F = rng.integers(220, 320, size=m)
            s = rng.integers(0, len(genome) - 320, size=m)
            r1 = genome[s[:, None] + np.arange(L)[None, :]]
            r2 = comp[genome[(s + F - L)[:, None] + np.arange(L)[None, :]][:, ::-1]]
            for r in (r1, r2):
                e = rng.random(r.shape) < 0.005
                r[e] = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=int(e.sum()))]
            for mate, (small, big) in enumerate(((reads0[2 * lo:2 * hi:2], r1), (reads0[2 * lo + 1:2 * hi:2], r2)),
                                                start=1):
                buf = fastq_bytes(f"c{c:04d}w", mate, small) + fastq_bytes(f"c{c:04d}b", mate, big)
                write_bgzf(os.path.join(cells_dir, f"cell{c:04d}_{mate}.fastq.gz"), buf, pool)
    t_gen = time.perf_counter() - t0
    outdir = os.path.join(folder, "out")
    t0 = time.perf_counter()
    merged = singlecell.run(paths["anchor"], cells_dir, paths["genome"], paths["gtf"], outdir, log=lambda *_: None)
    t_run = time.perf_counter() - t0
    rows = [k for k in merged.get("BCRX", {}) if "ABLX" in k]
    res = {
        "leg": "single cell: C BGZF FASTQ pairs -> singlecell.run (cells batched per GPU pass, S3-S8 per cell, "
               "SC:258-287 merge), one anchor",
        "cells": n_cells, "pairs_per_cell": per, "read_len": int(L),
        "wall_s": round(t_run, 3), "cells_per_s": round(n_cells / t_run, 2),
        "pairs_per_s": round(n_cells * per / t_run, 1),
        "fusion_rows": rows[:1], "cells_with_fusion": (merged["BCRX"][rows[0]][2] if rows else 0),
        "host_threads": int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count(),
        "generate_s": round(t_gen, 1), "truth_junction": truth["anchor_junction"],
    }
    line = json.dumps(res)
    print(line, flush=True)
    if out:
        with open(out, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
