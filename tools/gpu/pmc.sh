#!/bin/bash
# rocprofv3 PMC counter passes over graph-replayed training steps (256^2, B=16); one pass per counter group,
# each within the per-block slot limits (SQ 8, TCC 4 with FETCH_SIZE=3 / WRITE_SIZE=2). Summary: tools/pmc_summary.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out/pmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || echo "counter list failed"
cd /tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL ${PMC_T:-150} rocprofv3 --pmc $counters --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- \
      python $R/bench.py --profile-steps ${PSTEPS:-6} ${PROF_ARGS} > $R/gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "pass $i ($counters) failed rc=$rc"; tail -5 $R/gpurun_out/pmc/p$i.log; exit $rc; }
  echo "pass $i ok: $counters"
done < $R/${PMC_PASSES:-tools/pmc_passes.txt}
