#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over tools/one_pass.py for env settings.
#   PMC_RUNS="cfg4|SHDR_DEFER=0;cfg4|SHDR_DEFER=1"  PMC_GROUPS="SQ_WAVES SQ_WAVE_CYCLES ...;FETCH_SIZE"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
[ -n "$LIST" ] && { timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1; echo listed; }
IFS=';' read -ra RUNS <<< "$PMC_RUNS"
IFS=";" read -ra PGROUPS <<< "$PMC_GROUPS"
i=0
for r in "${RUNS[@]}"; do
  IFS='|' read -ra P <<< "$r"
  wl="${P[0]}"; envs="${P[1]}"
  j=0
  for grp in "${PGROUPS[@]}"; do
    d=gpurun_out/pmc/r${i}_g${j}
    echo "=== $wl [$envs] pmc: $grp"
    env $envs timeout -s KILL 200 rocprofv3 --pmc $grp -d $d -o run --output-format csv -- python3 tools/one_pass.py $wl 2 > $d.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 $d.log; exit 9; }
    j=$((j+1))
  done
  i=$((i+1))
done
python3 tools/summarize_pmc.py gpurun_out/pmc
