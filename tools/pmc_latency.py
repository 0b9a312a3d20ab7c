"""Per-kernel memory-latency view from rocprofv3 PMC passes (tools/pmc_latency_passes.txt via gpurun):

  L1->L2 lat TCP_TCC_READ_REQ_LATENCY_sum / TCP_TCC_READ_REQ_sum - average cycles of an L1 miss served by L2 / beyond
  L2 hit     TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  wait       SQ_WAIT_ANY / SQ_WAVE_CYCLES - share of wave time waiting on anything (memory, barriers, dependencies)
  vmem/wave  SQ_INSTS_VMEM / SQ_WAVES - vector-memory instructions per wave

    python tools/pmc_latency.py gpurun_out/pmc_lat [top]
"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_lat"
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    seen = set()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if "render_kernel" in k:
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), k, f)
        if key not in seen and f.endswith(os.path.join("p1", "run_counter_collection.csv")):
            seen.add(key)
            try:
                dur[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            except (KeyError, ValueError):
                pass


def ratio(c, a, b):
    return c[a] / c[b] if c.get(b) else float("nan")


print(f"{'kernel':58s} {'ms':>7s} {'L1>L2lat':>9s} {'L2hit':>6s} {'wait':>5s} {'vmem/wave':>9s}")
for k in sorted(tot, key=lambda k: -dur[k])[:top]:
    c = tot[k]
    vm = ratio(c, "SQ_INSTS_VMEM", "SQ_WAVES")
    l2 = ratio(c, "TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum")
    hit = c.get("TCC_HIT_sum", 0.0)
    miss = c.get("TCC_MISS_sum", 0.0)
    hr = hit / (hit + miss) if hit + miss else float("nan")
    wt = ratio(c, "SQ_WAIT_ANY", "SQ_WAVE_CYCLES")
    print(f"{k[:58]:58s} {dur[k] / 1e6:7.3f} {l2:9.0f} {100 * hr:5.1f}% {100 * wt:4.0f}% {vm:9.1f}")
