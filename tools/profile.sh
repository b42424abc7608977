#!/bin/bash
# rocprofv3 kernel trace + PMC passes (one counter group per pass, each its own
# run, as MI355X_MICROARCH.md prescribes) for one bench configuration, plus a
# FETCH_SIZE calibration pass over tools/ubench (known byte counts).
#   usage: tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/{ktrace,fetch,write,tcc,calib}; run from the repo root on the GPU box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
BENCH_ARGS=("$@")
run() {  # name, timeout, rocprof args... -- program...
  local name=$1 t=$2; shift 2
  echo "=== $(date +%T) $name"
  timeout -s KILL "$t" rocprofv3 "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== rc=$rc"
  [ $rc -eq 0 ] || exit 99
}
run ktrace 300 --kernel-trace --stats -d "$out/ktrace" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}"
run fetch 180 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}"
run write 180 --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}"
run tcc 180 --pmc TCC_HIT_sum TCC_MISS_sum -d "$out/tcc" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}"
if [ -x tools/ubench ]; then
  run calib 120 --pmc FETCH_SIZE -d "$out/calib" -o run --output-format csv -- ./tools/ubench 4096
fi
echo done
