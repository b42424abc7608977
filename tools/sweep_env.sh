#!/bin/bash
# One cfg4 bench run per environment setting: SETS="SHDR_DELTA=20 SHDR_DELTA=35 ..." (use , to join several vars).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sweep.log
for s in $SETS; do
  e=${s//,/ }
  env $e timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --no-cpu-baseline --no-side-configs $ARGS > gpurun_out/one.json 2>>gpurun_out/sweep.log || { echo "FATAL $s"; tail gpurun_out/sweep.log; exit 9; }
  echo -n "$s: "; python -c "import json;d=json.loads(open('gpurun_out/one.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],2),round(d['roofline']['kernel_ms'],2))"
done
