#!/bin/bash
# Same-box A/B of the working-tree library against libshdtopology_base.so (tools/build_base.sh):
# WL="cfg5 cfg4" REPS_LIB=2 BASE_ENV="SHDR_X=1"; optional GPU suite first (TESTS=1). Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
  tail -2 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; exit 1; }
fi
: > gpurun_out/ablib.log
for r in $(seq 1 ${REPS_LIB:-2}); do
  for wl in ${WL:-cfg5 cfg4}; do
    for lib in new base; do
      if [ $lib = base ]; then v=base; conf="${BASE_ENV:-}"; else v=""; conf="${NEW_ENV:-}"; fi
      echo "### rep $r $wl lib=$lib [$conf]" >> gpurun_out/ablib.log
      SHDR_LIB_VARIANT=$v REPS=1 PASSES=${PASSES:-2} timeout -k 10 300 python -u tools/ab.py $wl "$conf" >> gpurun_out/ablib.log 2>&1 || { echo "ab $wl $lib failed"; tail -20 gpurun_out/ablib.log; exit 9; }
    done
  done
done
grep -E "^###|warm mean" gpurun_out/ablib.log
