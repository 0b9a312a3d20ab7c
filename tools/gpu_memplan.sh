cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider -k memplan --timeout 240 --timeout-method thread > gpurun_out/memplan_test.log 2>&1 || { tail -30 gpurun_out/memplan_test.log; exit 1; }
tail -3 gpurun_out/memplan_test.log
timeout -k 10 600 python bench.py --img 512 --batch 0 --steps 1 --warmup 1 > gpurun_out/bench512.log 2>&1 || { tail -30 gpurun_out/bench512.log; exit 1; }
tail -2 gpurun_out/bench512.log
timeout -k 10 300 python bench.py --img 512 --batch 16 --steps 1 --warmup 1 --local-steps 100 > gpurun_out/bench512_b16.log 2>&1 || { tail -30 gpurun_out/bench512_b16.log; exit 1; }
tail -1 gpurun_out/bench512_b16.log
