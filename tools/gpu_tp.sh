#!/bin/bash
# Selected GPU tests (TEST_K), two bench runs, then a steady-state kernel trace (20 graph-replayed steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py} -x -q -m gpu -p no:cacheprovider --timeout 120 \
    --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps ${BSTEPS:-2} --warmup 1 $BENCH_ARGS > gpurun_out/bench_$i.log 2>&1 || { tail -20 gpurun_out/bench_$i.log; exit 1; }
  echo "bench $i: $(grep -o '"value": [0-9.]*' gpurun_out/bench_$i.log) $(grep -o '"ms_per_iteration": [0-9.]*' gpurun_out/bench_$i.log)"
done
rm -rf $R/gpurun_out/prof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- \
    python $R/bench.py --profile-steps 20 $BENCH_ARGS > $R/gpurun_out/prof.log 2>&1 || { tail -5 $R/gpurun_out/prof.log; exit 1; }
cd $R && python tools/prof_summary.py gpurun_out/prof | head -${PROF_LINES:-24}
