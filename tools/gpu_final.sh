#!/bin/bash
# Final evidence session, in two gpurun calls (one call is limited to 20 minutes):
#   STAGE=1  GPU suite + smoke, default bench line + rocprofv3 of it (cfg5)
#   STAGE=2  rocprofv3 of the cfg4 side line, strong-scaling proxy
# Each step under its own time limit; logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r04}
if [ "${STAGE:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -5 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 2; }
  tail -1 gpurun_out/smoke.log
  bash tools/gpu_evidence.sh $tag || exit 3
else
  bash tools/profile.sh ${tag}_cfg4 --workload cfg4 > gpurun_out/prof_cfg4.log 2>&1 || { tail gpurun_out/prof_cfg4.log; exit 4; }
  bash tools/gpu_proxy.sh || exit 5
fi
exit 0
