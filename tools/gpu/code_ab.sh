#!/bin/bash
# Same-box A/B of two source trees (code changes, not knobs): BASE = a built copy of another commit INSIDE the repo
# (e.g. `git worktree add -f abbase <commit>` + its own build_hip(); list `./abbase/build` in .gpurunignore), run
# interleaved with the current tree: REPS 256^2 bench pairs, R512 config-4 pairs, and one per-position kernel-trace
# diff (trace_diff.py). -> gpurun_out/${OUT:-code_ab}/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd); O=$R/gpurun_out/${OUT:-code_ab}; B=$R/${BASE:-abbase}
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
[ -f $B/bench.py ] || { echo "no base tree at $B"; exit 2; }
rm -rf $O; mkdir -p $O
cd /tmp
for v in base new; do
  d=$R; [ $v = base ] && d=$B
  timeout -k 10 240 rocprofv3 --kernel-trace -d $O/ta_$v -o run --output-format csv -- python $d/bench.py --profile-steps 20 \
      > $O/ta_$v.log 2>&1 || { tail -5 $O/ta_$v.log; exit 1; }
  f=$(find $O/ta_$v -name "*kernel_trace.csv" | head -1)
  [ "$f" = $O/ta_$v/run_kernel_trace.csv ] || mv "$f" $O/ta_$v/run_kernel_trace.csv
done
cd $R
python tools/trace_diff.py $O/ta_base $O/ta_new 1 > $O/trace_diff.txt; head -1 $O/trace_diff.txt
for i in $(seq ${REPS:-2}); do
  for v in base new; do
    d=$R; [ $v = base ] && d=$B
    (cd $d && timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $O/b256_$v.log 2>&1) || { tail -20 $O/b256_$v.log; exit 1; }
    echo "256 $v $(grep -o '"value": [0-9.]*' $O/b256_$v.log)" | tee -a $O/ab.txt
  done
done
for i in $(seq ${R512:-1}); do
  for v in base new; do
    d=$R; [ $v = base ] && d=$B
    (cd $d && timeout -k 10 400 python bench.py --img 512 --batch 0 --steps 2 --warmup 1 > $O/b512_$v.log 2>&1) || { tail -20 $O/b512_$v.log; exit 1; }
    echo "512 $v $(grep -o '"value": [0-9.]*' $O/b512_$v.log)" | tee -a $O/ab.txt
  done
done
