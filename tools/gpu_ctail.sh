#!/bin/bash
# cluster tail: bounds-checked parity, product suite, then whole-table and shard A/B (default vs clusters off)
set -o pipefail
mkdir -p gpurun_out
SHDR_LIB_VARIANT=bchk timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/ct_bchk.log 2>&1 || { echo bchk failed; tail -30 gpurun_out/ct_bchk.log; exit 1; }
tail -1 gpurun_out/ct_bchk.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ct.log 2>&1 || { echo product failed; tail -30 gpurun_out/ct.log; exit 1; }
tail -1 gpurun_out/ct.log
env REPS=2 timeout -k 10 300 python -u tools/ab.py cfg4 "" "SHDR_CLUSTER=1" > gpurun_out/ct_cfg4.log 2>&1 || { echo ab4 failed; tail -20 gpurun_out/ct_cfg4.log; exit 2; }
grep -A3 "== summary" gpurun_out/ct_cfg4.log
env REPS=1 timeout -k 10 300 python -u tools/ab.py cfg5 "" "SHDR_CLUSTER=1" > gpurun_out/ct_cfg5.log 2>&1 || { echo ab5 failed; tail -20 gpurun_out/ct_cfg5.log; exit 3; }
grep -A3 "== summary" gpurun_out/ct_cfg5.log
for n in 2 4; do
  env REPS=1 PART=$n PARTS_MAX=2 timeout -k 10 300 python -u tools/ab.py cfg5 "" "SHDR_CLUSTER=1" > gpurun_out/ct_cfg5_p$n.log 2>&1 || { echo ab5 $n failed; tail -20 gpurun_out/ct_cfg5_p$n.log; exit 4; }
  grep -A3 "== summary" gpurun_out/ct_cfg5_p$n.log
done
timeout -k 10 300 python -u tools/diag.py 4 cfg5 > gpurun_out/ct_diag_cfg5.log 2>&1 || { echo diag failed; tail -20 gpurun_out/ct_diag_cfg5.log; exit 5; }
grep -v amdgpu.ids gpurun_out/ct_diag_cfg5.log
