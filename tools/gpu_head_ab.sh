#!/bin/bash
# Head fwd / bwd timing vs grid cap (TUNE_HEAD_BLOCKS = 13): same-address metric / gradient atomics scale with the
# block count; then numerics tests for the head kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for cap in ${CAPS:-1024 512 256 128}; do
  timeout -k 10 120 python tools/kbench.py --ops head_fwd,head_bwd,grad_finish --reps 50 --tune 13=$cap \
      > gpurun_out/kb_head_$cap.log 2>&1 || { tail -20 gpurun_out/kb_head_$cap.log; exit 1; }
  echo "cap $cap"; grep -E "^ +[0-9.]+ +(head|grad)" gpurun_out/kb_head_$cap.log
done
echo done
