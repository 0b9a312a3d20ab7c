#!/bin/bash
# deterministic reduction mode: full GPU suite, then whole-bench A/B default vs --deterministic, then a trace A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { grep -E "^E |Error|FAILED|Timeout" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
VARIANTS="-;-- --deterministic" REPS=${REPS:-2} bash tools/gpu_bench_ab.sh || exit 1
if [ -n "$TRACE" ]; then VARIANTS="- -" PROF_ARGS="" bash tools/gpu_trace_ab.sh; fi
