#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a crash,
# abort, time limit or hang (exit codes 124/134/137/139 or negative), but let an
# ordinary test failure (pytest exit 1) continue to the next step.
#   usage: tools/gpu_step.sh <seconds> <logfile> <command...>
secs=$1; log=$2; shift 2
mkdir -p "$(dirname "$log")"
echo "=== $(date +%T) step: $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "=== $(date +%T) rc=$rc: $*" | tee -a gpurun_out/steps.log
tail -n 5 "$log"
case $rc in
  0|1) exit 0 ;;
  *) echo "FATAL step rc=$rc; stopping" | tee -a gpurun_out/steps.log; exit 99 ;;
esac
