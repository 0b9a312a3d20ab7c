#!/bin/bash
# Mixed weight-gradient launch A/B (tools/mix_probe.py): whole launch + each item alone, per VARIANTS entry
# (';'-separated CFL_MIX_TUNE strings, "-" = defaults). -> gpurun_out/wab/<i>.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp CFL_NO_JIT_BUILD=1
mkdir -p gpurun_out/wab
IFS=';' read -ra VS <<< "${VARIANTS:--}"
i=0
for v in "${VS[@]}"; do
  t=""; [ "$v" != "-" ] && t="$v"
  CFL_MIX_TUNE="$t" MIX_ALONE_ONLY=${ALONE_ONLY:-1} timeout -k 10 300 python tools/mix_probe.py ${IMG:-256} ${B:-16} \
      > gpurun_out/wab/$i.txt 2>&1 || { tail -20 gpurun_out/wab/$i.txt; exit 1; }
  echo "=== [$v]"; grep -v "amdgpu.ids" gpurun_out/wab/$i.txt | grep -v "^\[wgrad_mix\]" | head -40
  i=$((i+1))
done
