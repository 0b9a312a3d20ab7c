"""Steady-state training step of a ``rocprofv3 --kernel-trace`` run of ``bench.py --profile-steps N``, per kernel
POSITION: mean start offset in the step, duration and the idle gap before it (segmented at ``zero_spans_kernel``
as tools/prof_summary.py does).

    python tools/step_positions.py gpurun_out/prof_dir
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import csv  # noqa: E402
import collections  # noqa: E402


def main():
    d = sys.argv[1]
    path = os.path.join(d, "run_kernel_trace.csv")
    if not os.path.exists(path):
        import glob
        path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    tr = list(csv.DictReader(open(path)))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(tr) if "zero_spans_kernel" in r["Kernel_Name"]]
    segs = [(starts[i], starts[i + 1]) for i in range(1, len(starts) - 1)]
    mode = collections.Counter(b - a for a, b in segs).most_common(1)[0][0]
    segs = [(a, b) for a, b in segs if b - a == mode]
    names = [tr[segs[0][0] + k]["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
             for k in range(mode)]
    off = [0.0] * mode
    dur = [0.0] * mode
    gap = [0.0] * mode
    for a, _ in segs:
        t0 = int(tr[a]["Start_Timestamp"])
        prev_end = t0
        for k in range(mode):
            r = tr[a + k]
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            off[k] += (s - t0) / 1e3
            dur[k] += (e - s) / 1e3
            gap[k] += max(0, s - prev_end) / 1e3
            prev_end = e
    n = len(segs)
    walls = [(int(tr[b]["Start_Timestamp"]) - int(tr[a]["Start_Timestamp"])) / 1e3 for a, b in segs]
    print(f"{n} steady steps, {mode} kernels/step, wall {sum(walls) / n:.1f} us, busy {sum(dur) / n:.1f} us, "
          f"gaps {sum(gap) / n:.1f} us")
    print(f"{'pos':>3} {'start':>8} {'dur':>7} {'gap':>5}  kernel")
    for k in range(mode):
        print(f"{k:3d} {off[k] / n:8.1f} {dur[k] / n:7.1f} {gap[k] / n:5.1f}  {names[k][:110]}")


if __name__ == "__main__":
    main()
