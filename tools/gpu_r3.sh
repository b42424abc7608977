#!/bin/bash
# round-3 iteration session: GPU parity suite + smoke, quick cfg5/cfg4 bench lines,
# optional same-process A/B lines (AB="cfg5|ENV=a|ENV=b;cfg4|..."). Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $TESTS > gpurun_out/gpu_tests.log 2>&1; rc=$?
  tail -2 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit 1; }
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 9; }
  tail -1 gpurun_out/smoke.log
fi
for w in ${QUICK:-cfg5 cfg4}; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-side-configs --no-cpu-baseline --no-first-query > gpurun_out/quick_$w.log 2>&1 || { echo bench $w failed; tail -20 gpurun_out/quick_$w.log; exit 9; }
  python - gpurun_out/quick_$w.log <<'PY'
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(r["config"]["workload"][:5], "ms/step %.1f" % r["ms_per_step"], "pass %.1f" % r["roofline"]["kernel_ms"], "frac %.3f" % r["roofline"]["frac"], "cold %.1f" % r["cold"]["first_pass_kernel_ms"], r.get("layout"))
PY
done
if [ -n "$AB" ]; then
  IFS=';' read -ra LINES <<< "$AB"
  i=0
  for line in "${LINES[@]}"; do
    IFS='|' read -ra P <<< "$line"
    wl="${P[0]}"; confs=("${P[@]:1}")
    timeout -k 10 ${AB_TIMEOUT:-400} python -u tools/ab.py "$wl" "${confs[@]}" > gpurun_out/ab_$i.log 2>&1 || { echo "ab $wl failed"; tail -20 gpurun_out/ab_$i.log; exit 9; }
    grep -A20 "== summary" gpurun_out/ab_$i.log
    i=$((i+1))
  done
fi
if [ -n "$DIAG" ]; then
  timeout -k 10 400 python -u tools/diag.py 4 $DIAG > gpurun_out/diag.txt 2>&1 || { echo diag failed; tail gpurun_out/diag.txt; exit 9; }
  grep -v amdgpu.ids gpurun_out/diag.txt
fi
exit 0
