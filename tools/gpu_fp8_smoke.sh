cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "fp8" > gpurun_out/fp8_tests.log 2>&1 || { tail -30 gpurun_out/fp8_tests.log; exit 1; }
tail -1 gpurun_out/fp8_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --fp8 --steps 2 --warmup 1 > gpurun_out/bench_fp8.log 2>&1 || { tail -20 gpurun_out/bench_fp8.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_iteration": [0-9.]*\|"train_loss": [0-9.]*' gpurun_out/bench_fp8.log | tr '\n' ' '; echo
