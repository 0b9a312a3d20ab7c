#!/bin/bash
# Round-3 A/B driver: a pytest selection (TESTS, -k expression K), then the driver-style bench once per variant.
# VARIANTS: ';'-separated env assignments ("" = defaults), e.g. VARIANTS='CFL_HEAD_FUSE=0;;CFL_EVAL_CAP=128'.
# Each variant's JSON line goes to gpurun_out/ab3/<i>.json; a one-line summary per variant is printed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
O=gpurun_out/ab3
rm -rf $O; mkdir -p $O
if [ -n "${TESTS}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS} -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
      ${K:+-k "$K"} > $O/tests.log 2>&1 || { grep -E "^E |FAILED|Error" $O/tests.log | head -30; tail -3 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
IFS=';' read -ra VS <<< "${VARIANTS}"
[ ${#VS[@]} -eq 0 ] && VS=("")
i=0
for v in "${VS[@]}"; do
  timeout -k 10 300 env $v python bench.py ${BENCH_ARGS} > $O/$i.log 2>&1 || { echo "variant [$v] failed"; tail -20 $O/$i.log; exit 1; }
  grep '^{' $O/$i.log > $O/$i.json
  echo "[$v] $(grep -o '"value": [0-9.]*\|"ms_per_iteration": [0-9.]*' $O/$i.json | tr '\n' ' ')"
  i=$((i + 1))
done
