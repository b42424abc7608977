#!/bin/bash
# wave-model cluster rule: cluster parity (bounds-checked), then cfg4 shard A/B and the cfg5 8-way proxy
set -o pipefail
mkdir -p gpurun_out
SHDR_LIB_VARIANT=bchk timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tail_split or cluster or small_shard or partition" -x -v --timeout 120 --timeout-method thread > gpurun_out/acl_bchk.log 2>&1 || { echo bchk failed; tail -30 gpurun_out/acl_bchk.log; exit 1; }
tail -1 gpurun_out/acl_bchk.log
for n in 2 4 8; do
  env REPS=2 PART=$n timeout -k 10 300 python -u tools/ab.py cfg4 "" "SHDR_CLUSTER=1" "SHDR_CLUSTER=3" "SHDR_CLUSTER=4" > gpurun_out/acl_c4_p$n.log 2>&1 || { echo "c4 p$n failed"; tail -20 gpurun_out/acl_c4_p$n.log; exit 2; }
  grep -E "summary|\] cold mean" gpurun_out/acl_c4_p$n.log
done
env REPS=1 PART=8 timeout -k 10 300 python -u tools/ab.py cfg5 "" > gpurun_out/acl_c5_p8.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/acl_c5_p8.log; exit 3; }
grep -E "^rep" gpurun_out/acl_c5_p8.log
