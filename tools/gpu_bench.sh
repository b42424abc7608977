#!/bin/bash
# drop-in tests + the default bench line (driver command) on the box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dropin.log 2>&1 || { echo dropin failed; tail -30 gpurun_out/dropin.log; exit 1; }
tail -2 gpurun_out/dropin.log
s=$(date +%s)
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 9; }
echo "bench wall $(( $(date +%s) - s )) s"
tail -1 gpurun_out/bench.log
