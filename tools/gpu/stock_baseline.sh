#!/bin/bash
# Stock PyTorch-ROCm comparator (MIOpen) on the bench shapes: bf16 eager, bf16 hipGraph, fp32 eager.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "" "--graph" "--fp32"; do
  timeout -k 10 400 python tools/bench_torch_stock.py --img ${IMG:-256} --batch ${B:-16} --iters ${IT:-200} $a \
      >> gpurun_out/stock.log 2>&1 || { tail -20 gpurun_out/stock.log; exit 3; }
done
grep '^{' gpurun_out/stock.log
