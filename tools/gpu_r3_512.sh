#!/bin/bash
# Config 4 / 5 measurement at 512^2 with the HBM-planned batch: bench bf16, steady-state kernel trace,
# per-call roofline (kbench at batch 256: per-image throughput is saturated from 256 on) -> gpurun_out/$OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=${OUT:-r3_512}
O=$R/gpurun_out/$OUT
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p $O
for v in bf16; do
  A=""
  timeout -k 10 400 python bench.py --img 512 --batch 0 --steps 2 --warmup 1 $A > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  grep '^{' $O/bench_$v.log >> $O/bench.jsonl
  echo "$v: $(grep -o '"value": [0-9.]*' $O/bench_$v.log)"
done
cd /tmp
for v in bf16; do
  A=""
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- \
      python $R/bench.py --img 512 --batch 0 --profile-steps 6 $A > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  python $R/tools/prof_summary.py $O/prof_$v 50 > $O/summary_$v.txt || exit 1
  head -3 $O/summary_$v.txt
done
cd $R
timeout -k 10 500 python tools/kbench.py --img 512 --batch 256 --roofline --reps 5 > $O/roofline.txt 2>&1 || { tail -5 $O/roofline.txt; exit 1; }
tail -2 $O/roofline.txt
rm -rf $O/prof_*/run_kernel_trace.csv.gz
echo done
