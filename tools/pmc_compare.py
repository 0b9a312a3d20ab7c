"""Per-kernel PMC comparison of two rocprofv3 --pmc runs (e.g. the bf16 and the fp8 engine at 512^2): for every
kernel whose name contains FILTER (default "conv3x3"), summed over its dispatches:

  us/disp    mean dispatch duration in the counter pass
  TF/s       MFMA math rate: (SQ_INSTS_VALU_MFMA_MOPS_BF16 + SQ_INSTS_VALU_MFMA_MOPS_F8) * 512 flop / time
  MFMA busy  SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4): share of the SIMDs' busy cycles with the matrix pipe busy
  VALU/MFMA  SQ_INSTS_VALU / MFMA instructions (SQ_INSTS_VALU counts the MFMAs too)
  wait       SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls); waitany SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on waitcnt /
             barrier), activeany SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  LDS conf   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE

    python tools/pmc_compare.py gpurun_out/r5_fp8pmc/bf16 gpurun_out/r5_fp8pmc/fp8 [FILTER]
"""
import collections
import csv
import glob
import os
import sys


def load(d):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(lambda: collections.defaultdict(float))
    nd = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            if key not in nd[k][f]:
                nd[k][f].add(key)
                try:
                    dur[k][f] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                except (KeyError, ValueError):
                    pass
    return tot, dur, nd


def row(k, tot, dur, nd):
    c = tot[k]
    ts = [v for v in dur[k].values() if v > 0]
    t = sum(ts) / len(ts) if ts else 0.0
    n = max((len(v) for v in nd[k].values()), default=1)
    mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) + c.get("SQ_INSTS_VALU_MFMA_MOPS_F8", 0.0)
    tf = mops * 512 / t / 1e3 if t else 0.0
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, 4 * c.get("SQ_BUSY_CYCLES", 0.0))
    wc = max(1.0, c.get("SQ_WAVE_CYCLES", 0.0))
    lds = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0.0))
    mf = c.get("SQ_INSTS_MFMA", 0.0)
    valu = c.get("SQ_INSTS_VALU", 0.0) / mf if mf else float("nan")
    return (f"{t / n / 1e3:9.1f} {n:4d} {tf:8.1f} {100 * busy:6.1f}% {valu:7.1f} "
            f"{100 * c.get('SQ_WAIT_INST_ANY', 0.0) / wc:5.1f}% {100 * c.get('SQ_WAIT_ANY', 0.0) / wc:5.1f}% "
            f"{100 * c.get('SQ_ACTIVE_INST_ANY', 0.0) / wc:5.1f}% {100 * lds:5.1f}%  {k[:75]}")


def main():
    dirs = sys.argv[1:3]
    filt = sys.argv[3] if len(sys.argv) > 3 else "conv3x3"
    print("  us/disp disp     TF/s MFMAbusy VALU/MFMA  wait waitany actany LDSconf  kernel")
    for d in dirs:
        tot, dur, nd = load(d)
        print(f"== {d}")
        for k in sorted(tot, key=lambda k: -sum(dur[k].values())):
            if filt in k:
                print(row(k, tot, dur, nd))


if __name__ == "__main__":
    main()
