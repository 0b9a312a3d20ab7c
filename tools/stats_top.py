"""Top kernels of a rocprofv3 ``--stats`` run by total time (run_kernel_stats.csv).

    python tools/stats_top.py gpurun_out/evprof [top]
"""
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
paths = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
if not paths:
    sys.exit(f"no kernel_stats.csv under {d}")
skip = ("render_kernel", "FillFunctor", "copyBuffer")       # dataset render + harness fills
rows = [r for r in csv.DictReader(open(paths[0])) if not any(k in r["Name"] for k in skip)]
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{paths[0]}: {tot / 1e6:.3f} ms of kernels")
for r in rows[:top]:
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e3:10.1f} us {100 * t / tot:5.1f}% {int(r['Calls']):6d} calls {float(r['AverageNs']) / 1e3:9.1f} us  "
          f"{r['Name'][:110]}")
