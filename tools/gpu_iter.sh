#!/bin/bash
# One GPU iteration: kernel numerics tests -> per-op micro-benchmark at the bench shapes -> short bench.
# Stops at the first failing / crash-like step (each step under its own time limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kbench.py ${KBENCH_ARGS:---variants} > gpurun_out/kbench.log 2>&1
rc=$?
tail -40 gpurun_out/kbench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps ${BSTEPS:-3} --warmup 1 > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/bench.log
exit $rc
