#!/bin/bash
# rocprofv3 kernel trace + PMC passes for one bench configuration.
#   usage: tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/{ktrace,pmc_*}; run from the repo root on the GPU box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
run() {  # name, timeout, rocprof args...
  local name=$1 t=$2; shift 2
  echo "=== $(date +%T) $name"
  timeout -s KILL "$t" rocprofv3 "$@" -d "$out/$name" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== rc=$rc"
  [ $rc -eq 0 ] || exit 99
}
BENCH_ARGS=("$@")
run ktrace 300 --kernel-trace --stats
run fetch 180 --pmc FETCH_SIZE
run write 180 --pmc WRITE_SIZE
run tcc 180 --pmc TCC_HIT_sum TCC_MISS_sum
run sq 180 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS
echo done
