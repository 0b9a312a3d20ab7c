#!/bin/bash
# diag at a well-conditioned size + kernel-trace profile of 20 graph-replayed training steps (256^2, B=16)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_engine.py ${DIAG_S:-128} ${DIAG_B:-8} > gpurun_out/diag128.log 2>&1 || { tail -20 gpurun_out/diag128.log; exit 3; }
grep -E "^(grad|loss)" gpurun_out/diag128.log
grep -E "^param" gpurun_out/diag128.log | sort -k4 -n | head -8
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --profile-steps ${PSTEPS:-20} ${BENCH_ARGS} > $R/gpurun_out/prof.log 2>&1
rc=$?
tail -3 $R/gpurun_out/prof.log
find $R/gpurun_out/prof -name "*stats*" | head
exit $rc
