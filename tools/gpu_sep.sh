#!/bin/bash
# Knob A/B with one PROCESS per configuration (interleaved REPS_SEP times), for effects
# smaller than the same-process placement pattern: SEP="cfg5||SHDR_DELTA=18;cfg4||SHDR_X=1"
# (an empty field = defaults). Optional diagnostic-build breakdown afterwards: DIAG_RUNS
# as in tools/gpu_diag.sh. Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sep.log
IFS=';' read -ra LINES <<< "$SEP"
for r in $(seq 1 ${REPS_SEP:-2}); do
  for line in "${LINES[@]}"; do
    IFS='|' read -ra P <<< "$line"
    wl="${P[0]}"
    for conf in "${P[@]:1}"; do
      echo "### rep $r $wl [$conf]" >> gpurun_out/sep.log
      REPS=1 PASSES=${PASSES:-2} timeout -k 10 300 python -u tools/ab.py "$wl" "$conf" >> gpurun_out/sep.log 2>&1 || { echo "ab $wl [$conf] failed"; tail -20 gpurun_out/sep.log; exit 9; }
    done
  done
done
grep -E "^###|warm mean" gpurun_out/sep.log
if [ -n "$DIAG_RUNS" ]; then
  bash tools/gpu_diag.sh || exit 9
fi
exit 0
