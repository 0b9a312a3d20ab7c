#!/bin/bash
# GPU tests, then an A/B of bench.py under environment settings AB_VAR=each of AB_VALS, interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py} -x -q -m gpu -p no:cacheprovider --timeout 120 \
      --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
fi
V=${AB_VAR:-CFL_TUNE}
i=0
for rep in 1 2; do
  for val in ${AB_VALS:-"" "9=1"}; do
    i=$((i+1))
    env $V="$val" timeout -k 10 300 python bench.py --steps ${BSTEPS:-2} --warmup 1 $BENCH_ARGS > gpurun_out/ab_$i.log 2>&1 \
        || { tail -20 gpurun_out/ab_$i.log; exit 1; }
    echo "$V=$val rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/ab_$i.log) $(grep -o '"ms_per_iteration": [0-9.]*' gpurun_out/ab_$i.log)"
  done
done
