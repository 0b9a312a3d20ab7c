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

# busy vs wall over the graph-replayed steps (kernel trace): the gap share is launch/dependency overhead
import os  # noqa: E402
tp = f"{d}/run_kernel_trace.csv"
if os.path.exists(tp):
    tr = [r for r in csv.DictReader(open(tp)) if not any(s in r["Kernel_Name"] for s in skip)]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = len(tr)
    tail = tr[n // 2:]                       # second half: steady-state replays
    wall = int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail)
    print(f"steady state (last {len(tail)} kernels): wall {wall / 1e6:.3f} ms, kernel busy {busy / 1e6:.3f} ms, "
          f"idle {100 * (1 - busy / max(wall, 1)):.1f}%  (avg gap {(wall - busy) / 1e3 / max(len(tail) - 1, 1):.2f} us)")
