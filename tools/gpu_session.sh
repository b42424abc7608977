#!/bin/bash
# One GPU session: optional GPU suite, then same-box measurements, each step under
# its own time limit, logs under gpurun_out/. Steps are chained: the first failure ends it.
#   TESTS=1|0  run `pytest -m gpu` first (default 1)
#   STEPS      ';'-separated commands run after the suite (each: timeout 600)
set -o pipefail
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -1 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit 1; }
fi
i=0
IFS=';' read -ra cmds <<< "${STEPS:-}"
for c in "${cmds[@]}"; do
  [ -z "${c// }" ] && continue
  i=$((i+1))
  echo "### step $i: $c"
  eval "timeout -k 10 ${STEP_TIMEOUT:-600} $c" > gpurun_out/step_$i.log 2>&1 || { echo "step $i failed rc=$?"; tail -20 gpurun_out/step_$i.log; exit 9; }
  tail -8 gpurun_out/step_$i.log
done
exit 0
