#!/bin/bash
# A/B of an engine environment knob on the bench: ENVA vs ENVB (e.g. ENVA="SHDR_BUCKET_SORT=0"), cfg4 x N.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.log
run() { env $1 timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --no-cpu-baseline --no-side-configs $2 > gpurun_out/one.json 2>>gpurun_out/ab.log || { echo "FATAL"; tail gpurun_out/ab.log; exit 9; }; python -c "import json;d=json.loads(open('gpurun_out/one.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],2),round(d['roofline']['kernel_ms'],2),d['roofline']['kernel_ms_each'])"; }
for i in $(seq ${N:-2}); do
  echo -n "A [$ENVA]: "; run "$ENVA"
  echo -n "B [$ENVB]: "; run "$ENVB"
done
if [ -n "$CFG5" ]; then
  echo -n "cfg5 A: "; run "$ENVA" "--workload cfg5 --steps 1 --warmup 1"
  echo -n "cfg5 B: "; run "$ENVB" "--workload cfg5 --steps 1 --warmup 1"
fi
