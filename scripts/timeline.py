"""Timeline of the last bench step from a rocprofv3 kernel trace (profile_step.sh's kt/ directory):
per kernel name, the first start and last end relative to the step's start (the last trace
timestamp minus the step time), launches, and the summed busy time; the window's kernels sorted by
start.

usage: python3 scripts/timeline.py gpurun_out/<tag> [step_ms]
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:40]


def main():
    src = sys.argv[1]
    step_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 270.0
    f = glob.glob(os.path.join(src, "kt", "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in csv.DictReader(open(f))]
    end = max(e for _, e, _ in rows)
    t0 = end - int(step_ms * 1e6)
    win = [(s, e, k) for s, e, k in rows if e > t0]
    agg = collections.OrderedDict()
    for s, e, k in sorted(win):
        a = agg.setdefault(k, [s, e, 0, 0])
        a[1] = max(a[1], e)
        a[2] += 1
        a[3] += e - max(s, t0)
    print(f"window: last {step_ms} ms of the trace ({len(win)} dispatches)")
    print(f"{'kernel':40s} {'first_ms':>9s} {'last_ms':>9s} {'n':>5s} {'busy_ms':>9s}")
    for k, (s, e, n, b) in agg.items():
        print(f"{k:40s} {(s - t0) / 1e6:9.2f} {(e - t0) / 1e6:9.2f} {n:5d} {b / 1e6:9.2f}")


if __name__ == "__main__":
    main()
