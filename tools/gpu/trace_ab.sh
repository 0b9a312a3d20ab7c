#!/bin/bash
# Kernel-trace A/B of the steady-state step: one rocprofv3 --kernel-trace run of bench.py --profile-steps per
# variant (VARIANTS: space-separated --tune strings, "-" = default), then tools/trace_diff.py of each against the
# first. -> gpurun_out/ta/<i>/ (+ prof_summary of the first)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
rm -rf $R/gpurun_out/ta; mkdir -p $R/gpurun_out/ta
cd /tmp
i=0
for v in ${VARIANTS:--}; do
  t=""; [ "$v" != "-" ] && t="--tune $v"
  timeout -k 10 240 rocprofv3 --kernel-trace -d $R/gpurun_out/ta/$i -o run --output-format csv -- \
      python $R/bench.py --profile-steps ${PSTEPS:-20} $t ${PROF_ARGS} > $R/gpurun_out/ta/$i.log 2>&1 \
      || { tail -5 $R/gpurun_out/ta/$i.log; exit 1; }
  f=$(find $R/gpurun_out/ta/$i -name "*kernel_trace.csv" | head -1)
  [ "$f" = "$R/gpurun_out/ta/$i/run_kernel_trace.csv" ] || mv "$f" $R/gpurun_out/ta/$i/run_kernel_trace.csv
  i=$((i+1))
done
cd $R
python tools/prof_summary.py gpurun_out/ta/0 45 > gpurun_out/ta/summary0.txt && head -3 gpurun_out/ta/summary0.txt
j=0
for v in ${VARIANTS:--}; do
  if [ $j -gt 0 ]; then
    echo "=== [$v] vs default"
    python tools/trace_diff.py gpurun_out/ta/0 gpurun_out/ta/$j ${THR:-0.5}
  fi
  j=$((j+1))
done
find gpurun_out/ta -name "*.csv" ! -name "run_kernel_trace.csv" -delete
