#!/bin/bash
# validation (inference) kernel profile at the bench's eval batch: kernel stats of --profile-eval-steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
cd /tmp
rm -rf $R/gpurun_out/evprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/evprof -o run --output-format csv -- \
    python $R/bench.py --profile-eval-steps ${EVSTEPS:-12} > $R/gpurun_out/evprof.log 2>&1 || { tail -5 $R/gpurun_out/evprof.log; exit 1; }
cd $R && python tools/stats_top.py gpurun_out/evprof 25
