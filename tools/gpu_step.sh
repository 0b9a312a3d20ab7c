#!/bin/bash
# One measured iteration after a kernel change: every GPU test -> per-op timings of $OPS -> bench -> kernel-trace
# profile summary. Each GPU step under its own time limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
if [ -n "$OPS" ]; then
  timeout -k 10 180 python tools/kbench.py --ops $OPS --reps 50 > gpurun_out/kb_new.log 2>&1 \
      || { tail -20 gpurun_out/kb_new.log; exit 1; }
  sed -n '/per-op totals/,$p' gpurun_out/kb_new.log
fi
timeout -k 10 300 python bench.py --steps ${BSTEPS:-2} --warmup 1 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_iteration": [0-9.]*' gpurun_out/bench.log | tr '\n' ' '; echo
[ -n "$NOPROF" ] && { echo done; exit 0; }
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- \
    python $R/bench.py --profile-steps 20 > $R/gpurun_out/prof.log 2>&1 || { tail -5 $R/gpurun_out/prof.log; exit 1; }
cd $R && python tools/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.txt && head -14 gpurun_out/prof_summary.txt
echo done
