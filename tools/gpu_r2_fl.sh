#!/bin/bash
# FL product path + multi-rank rehearsal + overlapped FedAvg on the GPU (round-2 tests), then a short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fl.py "tests/test_gpu_kernels.py::test_overlapped_fedavg_bucket_repack_and_per_layer_waits" \
    -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -s > gpurun_out/gpu_fl.log 2>&1 \
    || { tail -60 gpurun_out/gpu_fl.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/gpu_fl.log | tail -8
