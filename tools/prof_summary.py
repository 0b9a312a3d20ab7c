"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel time per training step."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 21.0
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
skip = ("render_kernel",)
rows = [r for r in rows if not any(s in r["Name"] for s in skip)]
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"GPU kernel time per step: {tot / 1e6 / steps:.3f} ms  ({steps:.0f} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e6 / steps:8.3f} ms/step {100 * t / tot:6.2f}%  calls/step {int(r['Calls']) / steps:6.1f}  "
          f"avg {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:80]}")
