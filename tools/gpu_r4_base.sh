#!/bin/bash
# round-4 baseline: isolated 3x3 conv shapes under every variant + one driver-style bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/conv3_probe.py > gpurun_out/conv3_probe.txt 2>&1 || { tail -20 gpurun_out/conv3_probe.txt; exit 1; }
cat gpurun_out/conv3_probe.txt
timeout -k 10 400 python bench.py > gpurun_out/bench_base.log 2>&1 || { tail -20 gpurun_out/bench_base.log; exit 1; }
tail -1 gpurun_out/bench_base.log
