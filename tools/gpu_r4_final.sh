#!/bin/bash
# Round-4 final evidence bundle -> gpurun_out/r4_final: GPU suite, smoke, driver-style bench (x2) and the
# deterministic mode, steady-state kernel trace summary, per-call roofline, PMC passes + summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/r4_final
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || { grep -E "^E |Error|FAILED|Timeout" $O/gpu_tests.log | head -30; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 400 python bench.py > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  grep '^{' $O/bench_$i.log >> $O/bench.jsonl
done
timeout -k 10 400 python bench.py --deterministic > $O/bench_det.log 2>&1 || { tail -20 $O/bench_det.log; exit 1; }
grep '^{' $O/bench_det.log >> $O/bench.jsonl
grep -o '"value": [0-9.]*\|"deterministic": [a-z]*' $O/bench.jsonl | paste - - 
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python $R/bench.py --profile-steps 20 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $R
python tools/prof_summary.py $O/prof 50 > $O/summary_bf16.txt || exit 1
head -2 $O/summary_bf16.txt
rm -f $O/prof/*kernel_trace.csv*
timeout -k 10 400 python tools/kbench.py --roofline --reps 10 > $O/roofline.txt 2>&1 || { tail -5 $O/roofline.txt; exit 1; }
tail -2 $O/roofline.txt
if [ -z "$NO_PMC" ]; then
  bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc > $O/pmc_summary.txt && head -25 $O/pmc_summary.txt
fi
echo done
