#!/bin/bash
# partial-group-first: parity (bounds-checked build, then product), then the cfg5 8-way proxy
set -o pipefail
mkdir -p gpurun_out
SHDR_LIB_VARIANT=bchk timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tail_split or cluster or small_shard or partition" -x -v --timeout 120 --timeout-method thread > gpurun_out/pf_bchk.log 2>&1 || { echo bchk failed; tail -30 gpurun_out/pf_bchk.log; exit 1; }
tail -1 gpurun_out/pf_bchk.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tail_split" -x -v --timeout 120 --timeout-method thread > gpurun_out/pf.log 2>&1 || { echo product failed; tail -30 gpurun_out/pf.log; exit 1; }
tail -1 gpurun_out/pf.log
for n in 8 4 2; do
  env REPS=1 PART=$n timeout -k 10 300 python -u tools/ab.py cfg5 "" > gpurun_out/pf_p$n.log 2>&1 || { echo "p$n failed"; tail -20 gpurun_out/pf_p$n.log; exit 2; }
  grep "^rep" gpurun_out/pf_p$n.log
done
