#!/bin/bash
# Run a plan file on the GPU box: one command per line ('#' lines skipped), each under
# its own time limit (STEP_TIMEOUT, default 600 s), logs gpurun_out/<tag>_<i>.log.
# The first failing step ends the session (no retries).
#   usage: bash tools/gpu_plan.sh <planfile> [tag]
set -o pipefail
mkdir -p gpurun_out
plan=$1; tag=${2:-step}
i=0
while IFS= read -r c; do
  [ -z "${c// }" ] && continue
  [ "${c:0:1}" = "#" ] && continue
  i=$((i+1))
  echo "### $(date +%T) step $i: $c"
  eval "timeout -k 10 ${STEP_TIMEOUT:-600} $c" > gpurun_out/${tag}_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "step $i failed rc=$rc"; tail -25 gpurun_out/${tag}_$i.log; exit 9; fi
  tail -${TAIL:-6} gpurun_out/${tag}_$i.log
done < "$plan"
exit 0
