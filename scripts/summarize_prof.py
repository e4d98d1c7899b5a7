"""Turns a profile_step.sh output directory (gpurun_out/<tag>: kt/ kernel trace + stats, sq/ and
fetch/ counter passes of the configs[2] bench) into a round's committed profile summaries (profiles/rNN):

  kernel_stats_c3.csv   rocprofv3 --stats of the traced bench (3 timed + 1 warm-up steps)
  pmc_c3.json           per kernel of the step: launches, average duration (trace),
                                     VALU issue / wait / active fractions, resident waves, HBM
                                     FETCH_SIZE per launch (gfx950: x2 for wide reads), per unit
  pmc_c3.md             the same as a table

usage: python3 scripts/summarize_prof.py gpurun_out/<tag> profiles/rNN [bench_line.json]
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

CLOCK_GHZ = 2.4   # MI355X_MICROARCH.md: peak engine clock
N_SIMD = 1024     # 256 CUs x 4 SIMDs


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:60]


def main():
    src, out = sys.argv[1], sys.argv[2]
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    shutil.copy(stats[0], os.path.join(out, "kernel_stats_c3.csv"))
    dur = {}
    for r in csv.DictReader(open(stats[0])):
        k = short(r["Name"])
        c, t = dur.get(k, (0, 0.0))
        dur[k] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]))

    def counters(sub):
        acc = collections.defaultdict(float)
        disp = collections.defaultdict(dict)
        for f in glob.glob(os.path.join(src, sub, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                acc[(k, r["Counter_Name"])] += float(r["Counter_Value"])
                disp[k][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        avg = {k: v / len(disp[k[0]]) for k, v in acc.items()}
        ns = {k: sum(v.values()) / len(v) for k, v in disp.items()}
        return avg, {k: len(v) for k, v in disp.items()}, ns

    sq, nd, _ = counters("sq")
    fe, _, fe_ns = counters("fetch")
    wr, _, _ = counters("write") if os.path.isdir(os.path.join(src, "write")) else ({}, None, None)
    bench = {}
    if len(sys.argv) > 3 and os.path.exists(sys.argv[3]):
        bench = json.load(open(sys.argv[3]))
    counts = bench.get("counts_per_step", {})
    units = {  # units per launch of the step's kernels (bench counts per step)
        "k_g_seeds": ("genome reads (S4 + S5)", counts.get("queries_s4_s5")),
        "k_g_regions": ("genome reads (S4 + S5)", counts.get("queries_s4_s5")),
        "k_g_se": ("S5 split reads", counts.get("s5_split_reads")),
        "k_g_pe": ("S4 pairs", counts.get("s4_pairs")),
        "k_blat": ("S6 query strands", 2 * counts["s6_queries"] if counts.get("s6_queries") else None),
    }
    kern = {}
    for k in sorted(nd):
        g = lambda c: sq.get((k, c), 0.0)  # noqa: E731
        calls, tot = dur.get(k, (0, 0.0))
        avg_us = tot / calls / 1e3 if calls else None
        e = {"launches_counted": nd[k], "avg_duration_us": round(avg_us, 1) if avg_us else None}
        wc = g("SQ_WAVE_CYCLES")
        if wc:
            e["wait_any_frac"] = round(g("SQ_WAIT_ANY") / wc, 3)
            e["wait_inst_any_frac"] = round(g("SQ_WAIT_INST_ANY") / wc, 3)
            e["active_inst_frac"] = round(g("SQ_ACTIVE_INST_ANY") / wc, 3)
        if g("SQ_WAVES"):
            e["waves"] = int(g("SQ_WAVES"))
        # the counter pass's own duration in cycles: GRBM_GUI_ACTIVE sums the 8 XCDs
        # (MI355X_MICROARCH.md); SQ_WAVE_CYCLES / WAIT / ACTIVE count quad-cycles
        cyc = g("GRBM_GUI_ACTIVE") / 8
        if cyc:
            e["pmc_pass_cycles"] = round(cyc)
        if cyc and g("SQ_INSTS_VALU"):
            e["valu_per_launch"] = round(g("SQ_INSTS_VALU"))
            e["valu_issue_frac"] = round(g("SQ_INSTS_VALU") * 2 / (cyc * N_SIMD), 4)
        if cyc and wc:
            e["avg_resident_waves_per_simd"] = round(4 * wc / cyc / N_SIMD, 2)
        fs = fe.get((k, "FETCH_SIZE"))
        if fs is not None:
            e["fetch_bytes_per_launch_x2"] = round(fs * 1024 * 2)
            if fe_ns.get(k):  # over the FETCH pass's own dispatch time (kernels serialised)
                e["fetch_pass_us"] = round(fe_ns[k] / 1e3, 1)
                e["fetch_gbs_x2"] = round(fs * 1024 * 2 / fe_ns[k], 1)
        ws = wr.get((k, "WRITE_SIZE"))
        if ws is not None:  # WRITE_SIZE reads the bytes as they are (no gfx950 factor)
            e["write_bytes_per_launch"] = round(ws * 1024)
        for key, (uname, n) in units.items():
            if k.startswith(key) and n:
                e["unit"] = uname
                e["units_per_step"] = n
                if e.get("fetch_bytes_per_launch_x2") and calls:
                    e["fetch_bytes_per_unit_x2"] = round(e["fetch_bytes_per_launch_x2"] / n, 1)
                if e.get("write_bytes_per_launch") is not None and calls:
                    e["write_bytes_per_unit"] = round(e["write_bytes_per_launch"] / n, 1)
        kern[k] = e
    res = {"source": f"rocprofv3 --kernel-trace --stats, then --pmc passes (SQ; FETCH_SIZE; WRITE_SIZE) of "
                     f"python3 bench.py --no-cpu (configs[2], one GPU); {src}",
           "issue_model": "a wave64 VALU instruction issues over 2 cycles on a SIMD: valu_issue_frac = "
                          "SQ_INSTS_VALU x 2 / (pass cycles x 1024 SIMDs), pass cycles = GRBM_GUI_ACTIVE / 8 (the "
                          "counter pass's own dispatch, kernels serialised); resident waves = 4 x SQ_WAVE_CYCLES "
                          "(quad-cycles) / pass cycles / 1024; avg_duration_us is the kernel trace's (the step as "
                          "run: batches in flight, S4 beside S5 / S6)",
           "fetch_note": "FETCH_SIZE (KiB) x 1024 x 2: the gfx950 correction for wide coalesced reads; other "
                         "access widths are uncalibrated (MI355X_MICROARCH.md, HBM); GB/s over the FETCH pass's own "
                         "dispatch time",
           "kernels": kern}
    json.dump(res, open(os.path.join(out, "pmc_c3.json"), "w"), indent=1)
    cols = ["avg_duration_us", "fetch_pass_us", "pmc_pass_cycles", "valu_issue_frac", "wait_any_frac", "active_inst_frac",
            "avg_resident_waves_per_simd", "fetch_gbs_x2", "fetch_bytes_per_unit_x2", "write_bytes_per_unit"]
    lines = ["| kernel | " + " | ".join(cols) + " |", "|---" * (len(cols) + 1) + "|"]
    for k, e in kern.items():
        lines.append(f"| {k} | " + " | ".join(str(e.get(c, "")) for c in cols) + " |")
    open(os.path.join(out, "pmc_c3.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
