#!/bin/bash
# Same-box round-over-round A/B: the round-3 code (a git worktree of the round-3 verdict commit, built in-tree under
# _r3/) vs the current code, driver-style bench.py runs interleaved REPS times -> gpurun_out/r3r4/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/r3r4
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
rm -rf $O; mkdir -p $O
[ -d $R/_r3 ] || { echo "no _r3 worktree"; exit 1; }
for rep in $(seq 1 ${REPS:-3}); do
  (cd $R/_r3 && timeout -k 10 300 python bench.py > $O/r3_$rep.log 2>&1) || { tail -5 $O/r3_$rep.log; exit 1; }
  timeout -k 10 300 python bench.py > $O/r4_$rep.log 2>&1 || { tail -5 $O/r4_$rep.log; exit 1; }
  echo "rep $rep: r3 $(grep -o '"value": [0-9.]*' $O/r3_$rep.log)  r4 $(grep -o '"value": [0-9.]*' $O/r4_$rep.log)"
done
grep -h '^{' $O/r3_*.log > $O/bench_r3.jsonl
grep -h '^{' $O/r4_*.log > $O/bench_r4.jsonl
echo done
