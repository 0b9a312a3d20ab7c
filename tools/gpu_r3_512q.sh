#!/bin/bash
# Config 4 quick look: planned-batch bench (bf16) + steady-state kernel trace with per-call durations in step order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=${OUT:-r3_512q}
O=$R/gpurun_out/$OUT
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
rm -rf $O; mkdir -p $O
timeout -k 10 400 python bench.py --img 512 --batch 0 --steps 2 --warmup 1 ${BENCH_ARGS} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.jsonl
echo "bench: $(grep -o '"value": [0-9.]*' $O/bench.jsonl)"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python $R/bench.py --img 512 --batch 0 --profile-steps 4 ${BENCH_ARGS} > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python $R/tools/prof_summary.py $O/prof 50 > $O/summary_bf16.txt || exit 1
head -2 $O/summary_bf16.txt
echo done
