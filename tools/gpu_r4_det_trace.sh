#!/bin/bash
# Per-position kernel-trace A/B of the deterministic reduction mode against the default -> gpurun_out/r4_det
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/r4_det
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
rm -rf $O; mkdir -p $O
cd /tmp
i=0
for a in "" "--deterministic"; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d $O/$i -o run --output-format csv -- \
      python $R/bench.py --profile-steps 20 $a > $O/$i.log 2>&1 || { tail -5 $O/$i.log; exit 1; }
  f=$(find $O/$i -name "*kernel_trace.csv" | head -1)
  [ "$f" = "$O/$i/run_kernel_trace.csv" ] || mv "$f" $O/$i/run_kernel_trace.csv
  i=$((i+1))
done
cd $R
python tools/prof_summary.py $O/1 45 > $O/summary_det.txt && head -2 $O/summary_det.txt
python tools/trace_diff.py $O/0 $O/1 0.5 > $O/trace_diff.txt && head -40 $O/trace_diff.txt
rm -f $O/*/run_kernel_trace.csv
echo done
