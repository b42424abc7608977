#!/bin/bash
# Same-box interleaved A/B over (library flavour, engine knobs) pairs:
#   RUNS="prod|SHDR_PASS=1 prod|SHDR_PASS=0 split|" WL="cfg5 cfg4" REPS_LIB=2 PASSES=2 TAG=x
# ("prod" = libshdtopology.so, other names = libshdtopology_<name>.so; knobs space-separated
# after the bar, commas for several). One process per (rep, workload, run). Log: gpurun_out/abmix_<TAG>.log
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/abmix${TAG:+_$TAG}.log
: > "$L"
for r in $(seq 1 "${REPS_LIB:-2}"); do
  for wl in ${WL:-cfg5 cfg4}; do
    for run in $RUNS; do
      lib=${run%%|*}; conf=${run#*|}; conf=${conf//,/ }
      v=$lib; [ "$lib" = prod ] && v=""
      echo "### rep $r $wl lib=$lib [$conf]" >> "$L"
      SHDR_LIB_VARIANT=$v REPS=1 PASSES=${PASSES:-2} timeout -k 10 300 python -u tools/ab.py "$wl" "$conf" >> "$L" 2>&1 || { echo "ab $wl $run failed"; tail -20 "$L"; exit 9; }
    done
  done
done
python3 - "$L" <<'PY'
import re, sys, collections
cur = None; res = collections.defaultdict(list)
for l in open(sys.argv[1]):
    m = re.match(r"### rep \d+ (\S+) lib=(\S+) \[(.*)\]", l)
    if m: cur = (m.group(1), m.group(2), m.group(3)); continue
    m = re.search(r"warm mean ([\d.]+)", l)
    if m and cur: res[cur].append(float(m.group(1)))
for k, v in res.items():
    print(f"{k[0]:5s} {k[1]:8s} [{k[2]}] warm {' '.join(f'{x:.1f}' for x in v)}  mean {sum(v)/len(v):.1f}")
PY
