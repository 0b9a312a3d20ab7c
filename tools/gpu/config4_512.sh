#!/bin/bash
# Config 4 (512^2, planned batch) evidence -> gpurun_out/$OUT (default config4_512): bench (bf16, x2), steady-state kernel
# trace summary in step order, per-call roofline at batch 256
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/${OUT:-config4_512}
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
rm -rf $O; mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python bench.py --img 512 --batch 0 --steps 2 --warmup 1 > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  grep '^{' $O/bench_$i.log >> $O/bench.jsonl
done
grep -o '"value": [0-9.]*\|"global_batch": [0-9]*' $O/bench.jsonl | paste - -
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python $R/bench.py --img 512 --batch 0 --profile-steps 4 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $R
python tools/prof_summary.py $O/prof 50 > $O/summary_bf16.txt || exit 1
head -2 $O/summary_bf16.txt
rm -f $O/prof/*kernel_trace.csv*
timeout -k 10 400 python tools/kbench.py --img 512 --batch 256 --roofline --reps 5 > $O/roofline.txt 2>&1 || { tail -5 $O/roofline.txt; exit 1; }
tail -2 $O/roofline.txt
echo done
