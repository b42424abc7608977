#!/bin/bash
# GPU parity suite + smoke on the box; logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 9; }
tail -1 gpurun_out/smoke.log
