#!/bin/bash
# cluster-mode parity (bounds-checked build first, then the product build) and
# strong-scaling shard A/B; logs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
SHDR_LIB_VARIANT=bchk timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k cluster -x -v --timeout 120 --timeout-method thread > gpurun_out/cl_bchk.log 2>&1 || { echo bchk failed; tail -30 gpurun_out/cl_bchk.log; exit 1; }
tail -2 gpurun_out/cl_bchk.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k cluster -x -v --timeout 120 --timeout-method thread > gpurun_out/cl.log 2>&1 || { echo product failed; tail -30 gpurun_out/cl.log; exit 1; }
tail -2 gpurun_out/cl.log
[ "$1" = "tests" ] && exit 0
env REPS=2 PART=8 PARTS_MAX=3 timeout -k 10 300 python -u tools/ab.py cfg4 "" "SHDR_CLUSTER=2" "SHDR_CLUSTER=3" "SHDR_CLUSTER=4 SHDR_VARIANT=7" "SHDR_CLUSTER=2 SHDR_VARIANT=6" > gpurun_out/cl_ab_cfg4.log 2>&1 || { echo ab4 failed; tail -20 gpurun_out/cl_ab_cfg4.log; exit 2; }
tail -6 gpurun_out/cl_ab_cfg4.log
env REPS=1 PART=8 PARTS_MAX=2 timeout -k 10 400 python -u tools/ab.py cfg5 "" "SHDR_CLUSTER=2" "SHDR_CLUSTER=4" "SHDR_CLUSTER=4 SHDR_VARIANT=7" > gpurun_out/cl_ab_cfg5.log 2>&1 || { echo ab5 failed; tail -20 gpurun_out/cl_ab_cfg5.log; exit 3; }
tail -5 gpurun_out/cl_ab_cfg5.log
