#!/bin/bash
# GPU suite, then same-box A/B sweeps (tools/ab.py); everything logged under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit 1; }
i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "### $line"
  eval "timeout -k 10 600 $line" > gpurun_out/ab_$i.log 2>&1 || { echo "ab $i failed"; tail -5 gpurun_out/ab_$i.log; exit 9; }
  grep -A20 "== summary" gpurun_out/ab_$i.log
done < "${AB_PLAN:-tools/ab_plan.txt}"
