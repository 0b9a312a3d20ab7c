#!/bin/bash
# Per-kernel VGPR / occupancy / LDS / spill summary of a kernel TU (gfx950), from the compiler's resource remarks.
R=$(cd "$(dirname "$0")/.." && pwd)
for f in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I$R/csrc -I$R/csrc/kernels -c $R/csrc/kernels/$f.hip \
    -o /tmp/_ru.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip(); print(); print(cur[:90], end="")
    elif any(t.startswith(k) for k in ("VGPRs:", "AGPRs:", "Occupancy", "LDS Size", "VGPRs Spill", "ScratchSize")):
        print(" |", t.replace("[waves/SIMD]", "").replace("[bytes/block]", ""), end="")
print()'
done
