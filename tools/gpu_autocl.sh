#!/bin/bash
# automatic cluster rule: bounds-checked parity suite, product suite, then shard A/B (auto vs off)
set -o pipefail
mkdir -p gpurun_out
SHDR_LIB_VARIANT=bchk timeout -k 10 200 python -u tools/repro_cl.py "SHDR_CLUSTER=2" "SHDR_CLUSTER=4" > gpurun_out/acl_repro.log 2>&1; grep rep gpurun_out/acl_repro.log | cut -c1-60
SHDR_LIB_VARIANT=bchk timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/acl_bchk.log 2>&1 || { echo bchk failed; tail -30 gpurun_out/acl_bchk.log; exit 1; }
tail -1 gpurun_out/acl_bchk.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/acl.log 2>&1 || { echo product failed; tail -30 gpurun_out/acl.log; exit 1; }
tail -1 gpurun_out/acl.log
for n in 8 4 2; do
  env REPS=2 PART=$n PARTS_MAX=$n timeout -k 10 300 python -u tools/ab.py cfg4 "" "SHDR_CLUSTER=1" "SHDR_CLUSTER=2" "SHDR_CLUSTER=4" > gpurun_out/acl_cfg4_p$n.log 2>&1 || { echo ab4 $n failed; tail -20 gpurun_out/acl_cfg4_p$n.log; exit 2; }
  grep -A6 "== summary" gpurun_out/acl_cfg4_p$n.log
done
env REPS=1 PART=8 PARTS_MAX=3 timeout -k 10 300 python -u tools/ab.py cfg5 "" "SHDR_CLUSTER=1" > gpurun_out/acl_cfg5_p8.log 2>&1 || { echo ab5 failed; tail -20 gpurun_out/acl_cfg5_p8.log; exit 3; }
grep -A4 "== summary" gpurun_out/acl_cfg5_p8.log
