#!/bin/bash
# Steady-state profile of the default 256^2 / B16 step: driver-style bench line, rocprofv3 kernel trace of 20
# graph-replayed steps summarised per kernel (tools/prof_summary.py), per-call roofline (tools/kbench.py).
# -> gpurun_out/$OUT (copy the summaries worth keeping into profiles/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=${OUT:-r3_prof}
O=$R/gpurun_out/$OUT
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
rm -rf $O; mkdir -p $O
timeout -k 10 300 python bench.py ${BENCH_ARGS} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.jsonl
echo "bench: $(grep -o '"value": [0-9.]*\|"ms_per_iteration": [0-9.]*' $O/bench.jsonl | tr '\n' ' ')"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python $R/bench.py --profile-steps 20 ${PROF_ARGS} > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python $R/tools/prof_summary.py $O/prof 50 > $O/summary_bf16.txt || exit 1
head -3 $O/summary_bf16.txt
cd $R
if [ -z "${NO_ROOFLINE}" ]; then
  timeout -k 10 400 python tools/kbench.py --roofline --reps 10 > $O/roofline.txt 2>&1 || { tail -5 $O/roofline.txt; exit 1; }
  tail -2 $O/roofline.txt
fi
rm -f $O/prof/*kernel_trace.csv.gz
echo done
