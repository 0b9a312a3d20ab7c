#!/bin/bash
# sk A/B: kernel tests, probe, then whole-bench pairs default vs TUNE_CONV3_SK=3 (+ config override), eval profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
bash tools/gpu_sk.sh || exit 1
for v in "" "CONV3_SK=3" "" "CONV3_SK=3${SKCFG:+,CONV3_SK_CFG=$SKCFG}"; do
  timeout -k 10 300 python bench.py --steps 2 ${v:+--tune $v} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "bench [$v]: $(grep -o '"value": [0-9.]*' gpurun_out/ab.log) $(grep -o '"ms_per_iteration": [0-9.]*' gpurun_out/ab.log)"
done
CFL_EVAL_CAP=2048 timeout -k 10 300 python bench.py --steps 2 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
echo "bench [EVAL_CAP=2048]: $(grep -o '"value": [0-9.]*' gpurun_out/ab.log) $(grep -o '"eval_batch": [0-9]*' gpurun_out/ab.log)"
bash tools/gpu_r4_eval.sh
