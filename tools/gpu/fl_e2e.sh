#!/bin/bash
# End-to-end FL on the GPU box: server + 1 GPU client (HIP engine, hipGraph, evaluator) for 2 short rounds -> FIN,
# then a tensorboard/h5 artefact check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out/fl
timeout -k 10 400 python -m crack_detection_federatedlearning_grpc_amd.fl.launch --preset gpu1-256 \
    --max-rounds 2 --epochs 2 --steps-per-epoch 30 --synthetic-samples 1200 --val-samples 400 --predict-round 2 \
    --work-dir gpurun_out/fl --metrics-file gpurun_out/fl/metrics.jsonl --tensorboard --log-dir gpurun_out/fl/logs \
    --snapshot-dir gpurun_out/fl/snap > gpurun_out/fl/launch.log 2>&1 || { tail -30 gpurun_out/fl/launch.log; exit 1; }
grep -E "round|FIN|predict done|Evaluate" gpurun_out/fl/launch.log | tail -12
tail -2 gpurun_out/fl/metrics.jsonl
ls gpurun_out/fl/snap gpurun_out/fl/logs | head
