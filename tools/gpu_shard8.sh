#!/bin/bash
# cfg5 8-way shard (6,250 rows): bucket layout / cluster / variant A/B (tools/ab.py), logs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
env REPS=1 PART=8 PARTS_MAX=2 timeout -k 10 500 python -u tools/ab.py cfg5 "" "SHDR_VARIANT=2" "SHDR_CLUSTER=2" "SHDR_CLUSTER=4" "SHDR_BALANCE=1" "SHDR_CLUSTER_TAIL=1" "$@" > gpurun_out/shard8.log 2>&1 || { echo failed; tail -20 gpurun_out/shard8.log; exit 1; }
grep -E "summary|\] cold mean" gpurun_out/shard8.log
