#!/bin/bash
# conv3x3_sk iteration: its GPU tests (+ the 3x3 family) then the probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "3x3 or split_k" -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/sk_tests.log 2>&1 || { grep -E "^E |Error|FAILED|Timeout" gpurun_out/sk_tests.log | head -30; tail -3 gpurun_out/sk_tests.log; exit 1; }
tail -1 gpurun_out/sk_tests.log
PROBE_SK_ONLY=1 timeout -k 10 300 python -u tools/conv3_probe.py ${PROBE_RES:-16 32 64} > gpurun_out/conv3_probe_sk.txt 2>&1 || { tail -20 gpurun_out/conv3_probe_sk.txt; exit 1; }
cat gpurun_out/conv3_probe_sk.txt
