#!/bin/bash
# round-4 iteration: the 3x3 kernel tests, a kernel-trace A/B (TRACE_VARIANTS) and a whole-bench A/B (BENCH_VARIANTS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "${TEST_K:-3x3 or weight_stationary or split_k}" -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 \
    || { grep -E "^E |Error|FAILED|Timeout" gpurun_out/iter_tests.log | head -30; tail -3 gpurun_out/iter_tests.log; exit 1; }
tail -1 gpurun_out/iter_tests.log
if [ -n "$TRACE_VARIANTS" ]; then VARIANTS="$TRACE_VARIANTS" bash tools/gpu_trace_ab.sh || exit 1; fi
if [ -n "$BENCH_VARIANTS" ]; then VARIANTS="$BENCH_VARIANTS" bash tools/gpu_bench_ab.sh || exit 1; fi
