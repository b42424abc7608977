#!/bin/bash
# strong-scaling per-shard proxy (tools/ab.py, PART=N: every part of the partition
# timed, the job waits for the slowest), default engine (automatic cluster mode)
# against one workgroup per bucket (SHDR_CLUSTER=1). The full table is timed before
# and after the shards (box drift shows as a difference), and the efficiencies
# T(S) / (N * max part time) use their mean. Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
log=gpurun_out/proxy.log
: > $log
for wl in cfg4 cfg5; do
  echo "# $wl full" >> $log
  env REPS=1 timeout -k 10 200 python -u tools/ab.py $wl "" >> $log 2>&1 || { echo "full $wl failed"; tail -20 $log; exit 1; }
  for n in 2 4 8; do
    echo "# $wl PART=$n" >> $log
    env REPS=1 PART=$n timeout -k 10 300 python -u tools/ab.py $wl "" "SHDR_CLUSTER=1" >> $log 2>&1 || { echo "$wl $n failed"; tail -20 $log; exit 2; }
  done
  echo "# $wl full" >> $log
  env REPS=1 timeout -k 10 200 python -u tools/ab.py $wl "" >> $log 2>&1 || { echo "full $wl failed"; tail -20 $log; exit 1; }
done
grep -E "^#|summary|\] cold mean" $log
python3 - "$log" <<'PY'
import re, sys
cur = None; full = {}; part = {}
for l in open(sys.argv[1]):
    m = re.match(r"# (\S+) (full|PART=(\d+))", l)
    if m: cur = (m.group(1), int(m.group(3)) if m.group(3) else 0); continue
    m = re.match(r"\[(.*)\] cold mean [\d.]+\s+warm mean ([\d.]+)", l)
    if m and cur:
        if cur[1] == 0: full.setdefault(cur[0], []).append(float(m.group(2)))
        else: part.setdefault(cur, {})[m.group(1)] = float(m.group(2))
for (wl, n), d in sorted(part.items()):
    f = sum(full[wl]) / len(full[wl])
    auto = d.get("", float("nan")); plain = d.get("SHDR_CLUSTER=1", float("nan"))
    print(f"{wl} N={n}: full {' / '.join(f'{x:.1f}' for x in full[wl])} ms (mean {f:.1f}); slowest part {auto:.1f} ms (plain {plain:.1f}); "
          f"efficiency {f / (n * auto):.3f} (plain {f / (n * plain):.3f})")
PY
