#!/bin/bash
# GPU suite, then the rocprofv3 evidence session for the default bench line (tools/profile.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit 1; }
bash tools/profile.sh "$@"
