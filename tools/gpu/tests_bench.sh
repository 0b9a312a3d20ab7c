#!/bin/bash
# GPU check at HEAD: the whole gpu-marked test suite, then the driver-style 1-GPU bench (BSTEPS timed rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 ${TTIME:-900} python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --steps ${BSTEPS:-3} --warmup 1 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
