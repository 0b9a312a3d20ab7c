#!/bin/bash
# Config 4: U-Net 512^2 batch curve on one MI355X (per-client batch 256 / 512 / the HBM planner's, ~1016):
# images/s and peak HBM per client. One FL round per timed step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out/memplan
for b in 256 512 0; do
  timeout -k 10 400 python bench.py --img 512 --batch $b --steps 1 --warmup 1 > gpurun_out/memplan/b$b.log 2>&1 \
      || { tail -20 gpurun_out/memplan/b$b.log; exit 1; }
  grep '^{' gpurun_out/memplan/b$b.log >> gpurun_out/memplan/bench.jsonl
  echo "batch $b: $(grep -o '"value": [0-9.]*\|"peak_hbm_gb_per_client": [0-9.]*\|"per_client_batch": [0-9]*\|"ms_per_iteration": [0-9.]*' gpurun_out/memplan/b$b.log | tr '\n' ' ')"
done
