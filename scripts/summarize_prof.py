"""Turns a profile_bench.sh output directory into the committed profile summaries:
<out>/kernel_stats.csv (rocprofv3 --stats), <out>/pmc_summary.md and, for K1,
profiles/pmc_seed_filter.json (read by bench.py for roofline.traffic).

usage: python3 scripts/summarize_prof.py gpurun_out/<tag> profiles/<round>
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

src, out = sys.argv[1], sys.argv[2]
os.makedirs(out, exist_ok=True)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = {"k_seed_stream": "K1 k_seed_stream", "k_seed_ragged": "K1 k_seed_ragged", "k_align": "K2 k_align",
         "k_pairs": "K3 k_pairs"}


def short(name):
    if "k_align<" in name and ", true>" in name:
        return "K2 k_align (placement)"
    for k, v in SHORT.items():
        if k + "<" in name or k + "(" in name:
            return v
    return name.replace("(anonymous namespace)::", "").split("(")[0][:60]


stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
shutil.copy(stats[0], os.path.join(out, "kernel_stats.csv"))


def counters(sub):
    acc = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(src, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: v / len(disp[k[0]]) for k, v in acc.items()}, {k: len(v) for k, v in disp.items()}


fetch, nd = counters("pmc_fetch")
write, _ = counters("pmc_write")
sq, _ = counters("pmc_sq")
lines = ["# Counter summary (bench workload: 1 M 2x100 pairs, BCR anchor)", "",
         "Per-launch averages over the bench steps under rocprofv3 (separate `--pmc` passes).",
         "FETCH_SIZE/WRITE_SIZE are KiB; FETCH_SIZE is doubled for gfx950 wide reads (MI355X_MICROARCH.md, HBM).", "",
         "| kernel | launches | FETCH_SIZE KiB (raw) | fetched bytes (x2) | WRITE_SIZE KiB | written bytes |",
         "|---|---|---|---|---|---|"]
for k in sorted(nd):
    fs, ws = fetch.get((k, "FETCH_SIZE"), 0.0), write.get((k, "WRITE_SIZE"), 0.0)
    lines.append(f"| {k} | {nd[k]} | {fs:.1f} | {fs * 2048 / 1e6:.1f} MB | {ws:.1f} | {ws * 1024 / 1e6:.1f} MB |")
lines.append("")
for k in sorted(nd):
    vals = ", ".join(f"{c}={v:.4g}" for (kk, c), v in sorted(sq.items()) if kk == k)
    if vals:
        lines.append(f"- {k}: {vals}")
k1 = "K1 k_seed_stream"
fs, ws = fetch.get((k1, "FETCH_SIZE")), write.get((k1, "WRITE_SIZE"))
if fs is not None and ws is not None:
    hbm = int(fs * 2048 + ws * 1024)
    alg = 2_000_000 * 100 + 2_000_000 * 4
    lines += ["", f"K1 algorithmic bytes per launch: 2,000,000 reads x 100 B + 2,000,000 x int32 hits = {alg / 1e6:.1f} MB; "
              f"measured HBM-side traffic {hbm / 1e6:.1f} MB ({hbm / alg:.3f}x)."]
    json.dump({"kernel": "k_seed_stream (K1)", "pairs": 1000000, "read_len": 100,
               "source": f"{out} (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, bench.py --steps 3)",
               "fetch_size_kib_raw": round(fs, 2), "write_size_kib": round(ws, 2),
               "correction": "gfx950: FETCH_SIZE reports 1/2 of wide coalesced read bytes (MI355X_MICROARCH.md, HBM) -> x2; KiB -> bytes",
               "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg},
              open(os.path.join(ROOT, "profiles", "pmc_seed_filter.json"), "w"), indent=1)
open(os.path.join(out, "pmc_summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
