#!/bin/bash
# quick GPU iteration: kernel tests, 2 bench runs, optional kbench ops (KB_OPS) with roofline columns
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { grep -E "^E |Error|FAILED" gpurun_out/gpu_tests.log | head -20; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps ${BSTEPS:-2} --warmup 1 $BENCH_ARGS > gpurun_out/bench_$i.log 2>&1 || { tail -20 gpurun_out/bench_$i.log; exit 1; }
  echo "bench $i: $(grep -o '"value": [0-9.]*' gpurun_out/bench_$i.log) $(grep -o '"ms_per_iteration": [0-9.]*' gpurun_out/bench_$i.log)"
done
if [ -n "$KB_OPS" ]; then
  timeout -k 10 300 python tools/kbench.py --roofline --ops $KB_OPS --reps 20 > gpurun_out/kb.txt 2>&1 || { tail -5 gpurun_out/kb.txt; exit 1; }
  grep -A30 "per-op totals" gpurun_out/kb.txt
fi
