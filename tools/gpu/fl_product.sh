#!/bin/bash
# Product-path evidence -> gpurun_out/$OUT (default fl_product): FL product bench (gRPC server + client, HIP engine), a kernel
# trace of the 1-rank overlapped FedAvg path (tools/overlap_summary.py), and a short end-to-end FL launch to FIN
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/${OUT:-fl_product}
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
rm -rf $O; mkdir -p $O
timeout -k 10 500 python bench.py --fl --steps 2 --warmup 1 > $O/bench_fl.log 2>&1 || { tail -20 $O/bench_fl.log; exit 1; }
grep '^{' $O/bench_fl.log > $O/bench_fl.jsonl
grep -o '"value": [0-9.]*\|"metric": "[^"]*"' $O/bench_fl.jsonl | paste - -
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- \
    python $R/bench.py --fedavg-1rank --steps 3 --warmup 1 --local-steps 40 > $O/overlap.log 2>&1 || { tail -5 $O/overlap.log; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ "$f" = "$O/prof/run_kernel_trace.csv" ] || mv "$f" $O/prof/run_kernel_trace.csv
python tools/overlap_summary.py $O/prof > $O/overlap_summary.txt 2>&1 || { tail -5 $O/overlap_summary.txt; exit 1; }
tail -8 $O/overlap_summary.txt
rm -f $O/prof/run_kernel_trace.csv
mkdir -p $O/e2e
timeout -k 10 400 python -m crack_detection_federatedlearning_grpc_amd.fl.launch --preset gpu1-256 \
    --max-rounds 2 --epochs 2 --steps-per-epoch 30 --synthetic-samples 1200 --val-samples 400 \
    --work-dir $O/e2e --metrics-file $O/e2e/metrics.jsonl > $O/e2e/launch.log 2>&1 || { tail -30 $O/e2e/launch.log; exit 1; }
grep -E "round|FIN" $O/e2e/launch.log | tail -6
echo done
