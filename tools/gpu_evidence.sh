#!/bin/bash
# One evidence session: the default bench line (driver command), the rocprofv3 kernel
# trace + FETCH/WRITE/TCC passes of it (tools/profile.sh <tag>), then optional request-mix
# PMC passes (PMC_RUNS / PMC_GROUPS as tools/gpu_pmc.sh). Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r03}
s=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 9; }
echo "bench wall $(( $(date +%s) - s )) s"
tail -1 gpurun_out/bench.log
bash tools/profile.sh "$tag" || { echo "profile failed"; exit 9; }
if [ -n "$PMC_RUNS" ]; then bash tools/gpu_pmc.sh || exit 9; fi
exit 0
