#!/bin/bash
# Whole-bench A/B: driver-style bench.py runs of each variant, in REPS interleaved passes (run-to-run drift spreads
# over every variant). VARIANTS: ';'-separated list of "ENV=V ... -- bench args" (either side may be empty; "-" =
# the default). -> gpurun_out/bab/*.log, one summary line per run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out/bab
IFS=';' read -ra VS <<< "${VARIANTS:--}"
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for v in "${VS[@]}"; do
    envs="${v%%--*}"; args=""
    [[ "$v" == *--* ]] && args="${v#*--}"
    [ "$(echo $envs)" = "-" ] && envs=""
    log=gpurun_out/bab/v${i}_r${rep}.log
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-2} $args > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "[$v] r$rep: $(grep -o '"value": [0-9.]*' $log) $(grep -o '"ms_per_iteration": [0-9.]*' $log)"
    i=$((i+1))
  done
done
