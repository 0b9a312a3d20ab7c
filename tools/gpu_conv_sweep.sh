cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out
for t in "" "10=32" "9=2" "6=2"; do
  timeout -k 10 200 python tools/kbench.py --ops conv_igemm --reps 30 --tune "$t" > gpurun_out/kb_conv_$t.log 2>&1 || { tail -5 gpurun_out/kb_conv_$t.log; exit 1; }
done
paste gpurun_out/kb_conv_.log gpurun_out/kb_conv_10=32.log gpurun_out/kb_conv_9=2.log gpurun_out/kb_conv_6=2.log | awk -F'\t' '{printf "%-70s | %s | %s | %s\n", $1, substr($2,1,9), substr($3,1,9), substr($4,1,9)}' | head -60
