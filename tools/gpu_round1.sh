#!/bin/bash
# GPU check: kernel numerics tests, smoke, short bench. Stops at the first crash-like exit status.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export CFL_NO_JIT_BUILD=1
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --local-steps 50 > gpurun_out/bench_short.log 2>&1
rc=$?
cat gpurun_out/bench_short.log | tail -5
exit $rc
