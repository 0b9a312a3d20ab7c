#!/bin/bash
# One GPU iteration after a kernel change: numerics tests -> bench -> kernel-trace stats -> LDS/traffic counter pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps ${BSTEPS:-2} --warmup 1 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_iteration": [0-9.]*' gpurun_out/bench.log | tr '\n' ' '; echo
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- \
    python $R/bench.py --profile-steps 20 > $R/gpurun_out/prof.log 2>&1 || { tail -5 $R/gpurun_out/prof.log; exit 1; }
rm -rf $R/gpurun_out/pmc/p3; mkdir -p $R/gpurun_out/pmc
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/pmc/p3 -o run -- python $R/bench.py --profile-steps 6 > $R/gpurun_out/pmc/p3.log 2>&1 \
    || { tail -5 $R/gpurun_out/pmc/p3.log; exit 1; }
timeout -k 10 120 python $R/tools/graph_floor.py || exit 1
echo done
