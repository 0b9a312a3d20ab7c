#!/bin/bash
# rocprofv3 marker + kernel trace of a short FL round (roctx phase ranges from utils/trace.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1 CFL_ROCTX=1
mkdir -p gpurun_out
rm -rf gpurun_out/markers
cd /tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace -d $R/gpurun_out/markers -o run --output-format csv -- \
    python $R/bench.py --steps 1 --warmup 1 --epochs 2 --local-steps 50 > $R/gpurun_out/markers.log 2>&1 \
    || { tail -20 $R/gpurun_out/markers.log; exit 1; }
ls $R/gpurun_out/markers
python $R/tools/marker_summary.py $R/gpurun_out/markers
