#!/bin/bash
# rocprofv3 evidence for one bench configuration, in ONE session on the GPU box:
#   ktrace  --kernel-trace --stats of the bench command (its JSON line is kept too)
#   fetch / write / tcc   one PMC group per pass, each its own run (MI355X_MICROARCH.md)
#   calib   FETCH_SIZE over tools/ubench (known byte counts)
# plus the sha of the library sources the passes ran (routes.hip + host code), so a PMC summary is only ever used for
# the kernel it measured (bench.load_pmc_traffic checks it).
#   usage: tools/profile.sh <tag> [bench args...]     (run from the repo root on the box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
python3 -c "from shadow_amd.routes import src_kernel_sha; print(src_kernel_sha())" > "$out/kernel_sha"
BENCH_ARGS=(--no-cpu-baseline --no-first-query --no-side-configs "$@")
run() {  # name, timeout, rocprof args... -- program...
  local name=$1 t=$2; shift 2
  echo "=== $(date +%T) $name"
  timeout -s KILL "$t" rocprofv3 "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== rc=$rc"
  [ $rc -eq 0 ] || exit 99
}
run ktrace 300 --kernel-trace --stats -d "$out/ktrace" -o run --output-format csv -- python3 bench.py "${BENCH_ARGS[@]}"
run fetch 240 --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python3 bench.py "${BENCH_ARGS[@]}"
run write 240 --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- python3 bench.py "${BENCH_ARGS[@]}"
run tcc 240 --pmc TCC_HIT_sum TCC_MISS_sum -d "$out/tcc" -o run --output-format csv -- python3 bench.py "${BENCH_ARGS[@]}"
if [ -x tools/ubench ]; then
  run calib 120 --pmc FETCH_SIZE -d "$out/calib" -o run --output-format csv -- ./tools/ubench 4096
fi
grep '^{"metric"' "$out/ktrace.log" | tail -1 > "$out/bench_line.json"
echo done
