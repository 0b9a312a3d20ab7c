#!/bin/bash
# Launch-knob sweeps with the per-op micro-benchmark (one process per setting, each under its own limit).
# Usage: tools/gpu_sweep.sh OPS "tune1" "tune2" ...   e.g. tools/gpu_sweep.sh conv_wgrad "3=256" "3=768,4=2"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
ops=$1; shift
for t in "$@"; do
  echo "=== tune [$t] ops [$ops]" >> gpurun_out/sweep.log
  timeout -k 10 180 python tools/kbench.py --quiet --ops "$ops" --tune "$t" >> gpurun_out/sweep.log 2>&1 || exit $?
done
grep -E "===|total|calls" gpurun_out/sweep.log
