#!/bin/bash
# diagnostic-build phase breakdown under env settings: DIAG_RUNS="cfg4|SHDR_DEFER=0;cfg4|SHDR_DEFER=1;..."
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/diag.txt
IFS=';' read -ra RUNS <<< "$DIAG_RUNS"
for r in "${RUNS[@]}"; do
  IFS='|' read -ra P <<< "$r"
  wl="${P[0]}"; envs="${P[1]}"
  echo "### $wl $envs" >> gpurun_out/diag.txt
  env $envs timeout -k 10 300 python -u tools/diag.py 4 $wl >> gpurun_out/diag.txt 2>&1 || { echo "diag $wl $envs failed"; tail -20 gpurun_out/diag.txt; exit 9; }
done
grep -v amdgpu.ids gpurun_out/diag.txt
