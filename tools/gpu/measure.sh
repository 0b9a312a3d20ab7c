#!/bin/bash
# Full measurement pass at HEAD -> gpurun_out/$OUT: bench (bf16 x2), steady-state kernel trace,
# PMC counter passes, per-call roofline (kbench). Copy the summaries you keep into profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
OUT=${OUT:-measure}
O=$R/gpurun_out/$OUT
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p $O
for v in bf16; do
  A=""
  for i in 1 2; do
    timeout -k 10 300 python bench.py --steps 2 --warmup 1 $A > $O/bench_${v}_$i.log 2>&1 || { tail -20 $O/bench_${v}_$i.log; exit 1; }
    grep '^{' $O/bench_${v}_$i.log >> $O/bench.jsonl
    echo "$v $i: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$i.log)"
  done
done
cd /tmp
for v in bf16; do
  A=""
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- \
      python $R/bench.py --profile-steps 21 $A > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  python $R/tools/prof_summary.py $O/prof_$v 40 > $O/summary_$v.txt || exit 1
  head -3 $O/summary_$v.txt
done
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $counters --output-format csv -d $O/pmc/p$i -o run -- \
      python $R/bench.py --profile-steps 6 > $O/pmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_p$i.log; exit 1; }
done < $R/tools/pmc_passes.txt
python $R/tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt || exit 1
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $counters --output-format csv -d $O/pmc_lat/p$i -o run -- \
      python $R/bench.py --profile-steps 6 > $O/pmc_lat_p$i.log 2>&1 || { echo "latency pass $i failed"; tail -5 $O/pmc_lat_p$i.log; exit 1; }
done < $R/tools/pmc_latency_passes.txt
python $R/tools/pmc_latency.py $O/pmc_lat 40 > $O/pmc_latency.txt || exit 1
cd $R
timeout -k 10 400 python tools/kbench.py --roofline --reps 20 > $O/roofline.txt 2>&1 || { tail -5 $O/roofline.txt; exit 1; }
tail -2 $O/roofline.txt
rm -rf $O/prof_*/run_kernel_trace.csv.gz
echo done
