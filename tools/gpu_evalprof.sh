#!/bin/bash
# Kernel-trace profile of validation (inference) steps alone at the bench's eval batch, plus the FL phase split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
cd /tmp
rm -rf $R/gpurun_out/evprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/evprof -o run --output-format csv -- \
    python $R/bench.py --profile-eval-steps 37 > $R/gpurun_out/evprof.log 2>&1 || { tail -5 $R/gpurun_out/evprof.log; exit 1; }
cd $R && python tools/prof_summary.py gpurun_out/evprof 38 > gpurun_out/evprof_summary.txt && head -30 gpurun_out/evprof_summary.txt
echo done
