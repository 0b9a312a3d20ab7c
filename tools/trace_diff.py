"""Per-position comparison of two rocprofv3 --kernel-trace runs of ``bench.py --profile-steps N`` (same step
schedule, e.g. default vs a --tune variant): the steady-state step of each run (graph replays, segmented at
``zero_spans_kernel`` as in tools/prof_summary.py) averaged per kernel POSITION, then printed side by side with
the delta, so a variant that swaps one kernel for another shows where it gains or loses.

    python tools/trace_diff.py gpurun_out/ta/base gpurun_out/ta/var [min_abs_delta_us]
"""
import collections
import csv
import os
import sys


def steady(d):
    tr = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(tr) if "zero_spans_kernel" in r["Kernel_Name"]]
    segs = [(starts[i], starts[i + 1]) for i in range(1, len(starts) - 1)]
    mode = collections.Counter(b - a for a, b in segs).most_common(1)[0][0]
    segs = [(a, b) for a, b in segs if b - a == mode]
    names = [tr[segs[0][0] + k]["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
             for k in range(mode)]
    t = [0.0] * mode
    for a, _ in segs:
        for k in range(mode):
            r = tr[a + k]
            t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    walls = [(int(tr[b]["Start_Timestamp"]) - int(tr[a]["Start_Timestamp"])) / 1e3 for a, b in segs]
    return names, [x / len(segs) for x in t], sum(walls) / len(walls)


def main():
    a, b = sys.argv[1], sys.argv[2]
    thr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
    na, ta, wa = steady(a)
    nb, tb, wb = steady(b)
    print(f"step wall: {wa:8.1f} us ({len(na)} kernels)  vs  {wb:8.1f} us ({len(nb)} kernels)  delta {wb - wa:+.1f}")
    if len(na) != len(nb):
        print("different kernel counts: per-position comparison up to the shorter step")
    for k in range(min(len(na), len(nb))):
        d = tb[k] - ta[k]
        if abs(d) >= thr or na[k] != nb[k]:
            print(f"{k:3d} {ta[k]:7.1f} {tb[k]:7.1f} {d:+6.1f}  {na[k][:70]}"
                  + (f"  ->  {nb[k][:70]}" if na[k] != nb[k] else ""))
    print(f"kernel sum: {sum(ta):.1f} vs {sum(tb):.1f} us")


if __name__ == "__main__":
    main()
