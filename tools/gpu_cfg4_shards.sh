#!/bin/bash
# cfg4 2- and 4-way shards: bucket layout A/B (tools/ab.py, every part timed), logs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
for n in 4 2; do
  env REPS=2 PART=$n timeout -k 10 300 python -u tools/ab.py cfg4 "" "SHDR_CLUSTER=2" "SHDR_CLUSTER=3" "SHDR_BALANCE=1" "SHDR_VARIANT=6" "SHDR_VARIANT=6 SHDR_BALANCE=1" > gpurun_out/c4_p$n.log 2>&1 || { echo "p$n failed"; tail -20 gpurun_out/c4_p$n.log; exit 2; }
  grep -E "summary|\] cold mean" gpurun_out/c4_p$n.log
done
