#!/bin/bash
# strong-scaling per-shard proxy (tools/ab.py, PART=N: every part of the partition
# timed, the job waits for the slowest), default engine (automatic cluster mode)
# against one workgroup per bucket (SHDR_CLUSTER=1); logs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
log=gpurun_out/proxy.log
: > $log
for wl in cfg4 cfg5; do
  env REPS=1 timeout -k 10 200 python -u tools/ab.py $wl "" >> $log 2>&1 || { echo "full $wl failed"; tail -20 $log; exit 1; }
  for n in 2 4 8; do
    echo "# $wl PART=$n" >> $log
    env REPS=1 PART=$n timeout -k 10 300 python -u tools/ab.py $wl "" "SHDR_CLUSTER=1" >> $log 2>&1 || { echo "$wl $n failed"; tail -20 $log; exit 2; }
  done
done
grep -E "^#|summary|\] cold mean" $log
