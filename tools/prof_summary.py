"""Summarise a rocprofv3 --kernel-trace run of ``bench.py --profile-steps N``: per-kernel time per STEADY-STATE step.

The trace holds the dataset render kernels, the eager warm-up step that precedes graph capture and N graph replays.
Steps are delimited by ``zero_spans_kernel`` (the first kernel of every training step); the summary drops everything
before the second step start (render + eager warm-up) and averages over the remaining graph-replayed steps only:
kernel time per step by kernel, step wall-clock (zero_spans start to the next one) and the idle share between kernels.

    python tools/prof_summary.py gpurun_out/prof [top]
"""
import collections
import csv
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
path = os.path.join(d, "run_kernel_trace.csv")
tr = list(csv.DictReader(open(path)))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(tr) if "zero_spans_kernel" in r["Kernel_Name"]]
if len(starts) < 3:
    sys.exit(f"{path}: fewer than 3 training steps in the trace")
# steps = zero_spans-to-zero_spans segments from the first graph replay on (step 0 = eager warm-up); segments whose
# kernel count differs from the typical step's (extra eager / calibration launches, e.g. the fp8 path's amax warm-up
# before its capture) are left out, so the figures describe graph-replayed steps only
segs = [(starts[i], starts[i + 1] if i + 1 < len(starts) else len(tr)) for i in range(1, len(starts))]
mode = collections.Counter(b - a for a, b in segs[:-1] or segs).most_common(1)[0][0]
segs = [(a, b) for a, b in segs if b - a == mode or (b == len(tr) and b - a >= mode)]
nsteps = len(segs)
steady = [r for a, b in segs for r in tr[a:a + mode]]
walls = [(int(tr[b]["Start_Timestamp"]) if b < len(tr) else int(tr[a + mode - 1]["End_Timestamp"]))
         - int(tr[a]["Start_Timestamp"]) for a, b in segs]
per = collections.defaultdict(lambda: [0, 0])
busy = 0
for r in steady:
    t = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    per[name][0] += t
    per[name][1] += 1
    busy += t
wall = sum(walls)
print(f"steady state: {nsteps} graph-replayed steps (eager warm-up + dataset render excluded)")
print(f"step wall-clock {wall / nsteps / 1e3:.1f} us (min {min(walls) / 1e3:.1f}, max {max(walls) / 1e3:.1f}); "
      f"kernel busy {busy / nsteps / 1e3:.1f} us/step; idle between kernels {100 * (1 - busy / wall):.1f}%; "
      f"{len(steady) / nsteps:.0f} kernels/step")
print(f"{'us/step':>9} {'share':>6} {'calls':>6} {'avg us':>8}  kernel")
for name, (t, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{t / nsteps / 1e3:9.1f} {100 * t / busy:5.1f}% {n / nsteps:6.1f} {t / n / 1e3:8.1f}  {name[:90]}")
