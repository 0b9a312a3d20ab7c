"""Per-kernel summary of the rocprofv3 PMC passes written by tools/gpu/pmc.sh (gpurun_out/pmc/p*/).

Per kernel (all dispatches of one kernel name, over the profiled steps):
  time       sum of dispatch durations in the pass (counter collection serialises dispatches)
  MFMA TF/s  SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 flop / time, and % of the 2.5 PFLOP/s dense bf16 peak
  HBM GB/s   (2 * FETCH_SIZE + WRITE_SIZE) KiB / time  (FETCH_SIZE counts half of a wide coalesced read on gfx950)
  LDS conf   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait       SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue-stall share of wave time)
"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
tot = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    seen = set()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if "render_kernel" in k:
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), k)
        if key not in seen:
            seen.add(key)
            try:
                dur[k][f] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            except (KeyError, ValueError):
                pass


def t_ns(k):
    v = [x for x in dur[k].values() if x > 0]
    return sum(v) / len(v) if v else 0.0


rows = sorted(tot, key=lambda k: -t_ns(k))
print(f"{'kernel':58s} {'ms':>7s} {'MFMA TF/s':>9s} {'%peak':>6s} {'HBM GB/s':>8s} {'LDSconf':>7s} {'wait':>5s}")
for k in rows:
    c, t = tot[k], t_ns(k)
    if t <= 0:
        continue
    fl = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) * 512
    tf = fl / t / 1e3                                       # flop/ns = GFLOP/s -> /1e3 TFLOP/s
    hbm = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / t   # bytes/ns = GB/s
    lds = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 0), 1)
    wait = c.get("SQ_WAIT_INST_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 0), 1)
    print(f"{k[:58]:58s} {t / 1e6:7.3f} {tf:9.1f} {100 * tf / 2500:6.1f} {hbm:8.0f} "
          f"{100 * lds:6.1f}% {100 * wait:4.0f}%")
