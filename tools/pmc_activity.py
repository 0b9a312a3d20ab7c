"""Per-kernel instruction-issue activity from a pass over SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES (rocprofv3 --pmc CSV):
SQ_ACTIVE_INST_{VALU,LDS,ANY} / SQ_WAVE_CYCLES = the share of a wave's resident cycles in which it issued that
instruction class (MFMA issue counts as VALU). Low ANY with high wait means the kernel is latency-bound.

usage: python tools/pmc_activity.py <pmc dir with run_counter_collection.csv> [top]
"""
import collections
import csv
import glob
import os
import sys


def main() -> int:
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    rows = []
    for k, c in agg.items():
        if k.startswith("render_kernel"):
            continue
        wc = c["SQ_WAVE_CYCLES"] or 1.0
        rows.append((c["GRBM_GUI_ACTIVE"], k, len(disp[k]), c["SQ_ACTIVE_INST_VALU"] / wc,
                     c["SQ_ACTIVE_INST_LDS"] / wc, c["SQ_ACTIVE_INST_ANY"] / wc))
    rows.sort(reverse=True)
    print(f"{'kernel':60s} {'calls':>5s} {'VALU':>6s} {'LDS':>6s} {'ANY':>6s}   (issue share of wave cycles)")
    for _, k, n, v, l, a in rows[:top]:
        print(f"{k:60s} {n:5d} {v:6.3f} {l:6.3f} {a:6.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
