#!/bin/bash
# Round-end rehearsal: the whole GPU test suite (one process), smoke(), then the driver's default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_all.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/gpu_all.log | head -30; tail -3 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
