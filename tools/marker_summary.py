"""Kernel time per roctx phase range from a rocprofv3 --marker-trace --kernel-trace run (tools/gpu/markers.sh).

A kernel belongs to the innermost range whose host push/pop interval contains the kernel's dispatch (correlation)
on the host side; graph replays are attributed by their launch time, so the GPU work of an asynchronously enqueued
phase may trail its range - totals per range are therefore reported as kernel busy time by launch window."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/markers"
mk = glob.glob(os.path.join(d, "*marker_api_trace.csv"))
kt = glob.glob(os.path.join(d, "*kernel_trace.csv"))
if not mk or not kt:
    print("missing marker or kernel trace in", d, os.listdir(d))
    sys.exit(0)
ranges = [r for r in csv.DictReader(open(mk[0]))]
print(f"{len(ranges)} marker records; columns: {list(ranges[0].keys()) if ranges else []}")
names = collections.Counter(r.get("Message") or r.get("Function") or "" for r in ranges)
print("ranges:", dict(names))
kern = list(csv.DictReader(open(kt[0])))
spans = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Message") or r.get("Function", "")) for r in ranges
         if r.get("Start_Timestamp") and r.get("End_Timestamp")]
tot = collections.defaultdict(float)
cnt = collections.Counter()
for k in kern:
    s0, e0 = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    inside = [sp for sp in spans if sp[0] <= s0 <= sp[1]]
    name = min(inside, key=lambda sp: sp[1] - sp[0])[2] if inside else "(outside)"
    tot[name] += (e0 - s0) / 1e6
    cnt[name] += 1
for n in sorted(tot, key=lambda n: -tot[n]):
    print(f"{n:28s} {cnt[n]:7d} kernels {tot[n]:10.3f} ms GPU")
