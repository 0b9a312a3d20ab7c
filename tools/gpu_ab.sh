#!/bin/bash
# GPU tests, then an A/B of bench.py under two environment settings (AB_VAR=0 / 1), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 \
      --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
V=${AB_VAR:-CFL_WGRAD_STREAM}
for rep in 1 2; do
  for val in ${AB_VALS:-0 1}; do
    env $V=$val timeout -k 10 300 python bench.py --steps ${BSTEPS:-2} --warmup 1 $BENCH_ARGS > gpurun_out/ab_${val}_$rep.log 2>&1 \
        || { tail -20 gpurun_out/ab_${val}_$rep.log; exit 1; }
    echo "$V=$val rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/ab_${val}_$rep.log) $(grep -o '"ms_per_iteration": [0-9.]*' gpurun_out/ab_${val}_$rep.log)"
  done
done
