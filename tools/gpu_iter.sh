#!/bin/bash
# iteration session: GPU parity suite, quick cfg5/cfg4 bench lines, optional diag
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit 1; }
for w in cfg5 cfg4; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-side-configs --no-cpu-baseline --no-first-query > gpurun_out/quick_$w.log 2>&1 || { echo bench $w failed; tail -20 gpurun_out/quick_$w.log; exit 9; }
  python - gpurun_out/quick_$w.log <<'PY'
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(r["config"]["workload"][:5], "ms/step %.1f" % r["ms_per_step"], "pass %.1f" % r["roofline"]["kernel_ms"], "frac %.3f" % r["roofline"]["frac"], "cold %.1f" % r["cold"]["first_pass_kernel_ms"])
PY
done
if [ -n "$DIAG" ]; then
  timeout -k 10 400 python -u tools/diag.py 4 $DIAG > gpurun_out/diag.txt 2>&1 || { echo diag failed; tail gpurun_out/diag.txt; exit 9; }
  cat gpurun_out/diag.txt | grep -v amdgpu.ids
fi
