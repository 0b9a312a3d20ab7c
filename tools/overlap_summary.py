"""Overlap of the FedAvg side stream with the compute stream, from a rocprofv3 kernel trace of
``bench.py --fedavg-1rank`` (or any N-rank bench run).

FedAvgAllReduce.average_async issues each bucket's all-reduce (RCCL kernels on RCCL's stream; bucket 0 = the
encoder's parameters) and then, on the aggregation side stream, that bucket's bf16 repack (pack_kernel); the next
round's first training step replays its two split graphs (UNetEngine.train_step): the encoder graph after bucket 0,
the rest of the step after every bucket. Per FL-round boundary this reports the side-queue busy time
(RCCL + side-stream pack kernels), how much of it ran while a compute-queue kernel was running (overlap fraction), and
the compute-queue idle time inside that window.

    python tools/overlap_summary.py gpurun_out/overlap/prof
"""
import csv
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/overlap/prof"
tr = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in tr]
rccl = [x for x in iv if "nccl" in x[3].lower() or "rccl" in x[3].lower()]
if not rccl:
    print("no RCCL kernels in the trace: a 1-rank all-reduce launches none (the overlap exists only at N > 1)")
side_q = {x[2] for x in rccl}
# the per-bucket repacks run on the aggregation side stream: pack kernels on a queue other than the compute queue
count = {}
for x in iv:
    count[x[2]] = count.get(x[2], 0) + 1
compute_q = max(count, key=count.get)
# the aggregation path = RCCL kernels + the per-bucket repacks (pack_kernel) NOT on the compute queue; other
# side-queue work (torch fills / copies of the harness) is not part of it
side = [x for x in iv if x[2] != compute_q and (x in rccl or "pack_kernel" in x[3])]
comp = [x for x in iv if x[2] == compute_q]


def union(xs):
    out = []
    for a, b, *_ in sorted(xs):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inter(u, v):
    i = j = tot = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            tot += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return tot


us, uc = union(side), union(comp)
busy_side = sum(b - a for a, b in us)
ov = inter(us, uc)
win = (us[0][0], us[-1][1]) if us else (0, 0)
comp_in_win = inter(uc, [list(win)])
print(f"compute queue {compute_q}: {len(comp)} kernels; side queues {sorted({x[2] for x in side})} "
      f"(RCCL on {sorted(side_q)}): {len(side)} kernels ({len(rccl)} RCCL)")
print(f"side-stream busy {busy_side / 1e3:.1f} us, of which {ov / 1e3:.1f} us overlapped compute-queue kernels: "
      f"overlap fraction {100 * ov / max(busy_side, 1):.1f}%")
print(f"window first->last side kernel {(win[1] - win[0]) / 1e3:.1f} us; compute busy inside it "
      f"{comp_in_win / 1e3:.1f} us")
names = {}
for x in side:
    k = x[3].split("(")[0][:60]
    names[k] = names.get(k, 0) + (x[1] - x[0])
for k, t in sorted(names.items(), key=lambda kv: -kv[1])[:8]:
    print(f"  side {t / 1e3:8.1f} us  {k}")
