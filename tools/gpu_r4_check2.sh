#!/bin/bash
# round-4 check at HEAD: full GPU test suite, smoke, driver-style bench, steady-state kernel trace summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { grep -E "^E |Error|FAILED|Timeout" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_check.log 2>&1 || { tail -20 gpurun_out/bench_check.log; exit 1; }
grep "^{" gpurun_out/bench_check.log | cut -c1-300
VARIANTS="-" bash tools/gpu_trace_ab.sh
