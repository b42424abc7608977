set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 3 --warmup 1 --no-side-configs --no-cpu-baseline > gpurun_out/base_cfg5.log 2>&1 || { echo cfg5 failed; tail -20 gpurun_out/base_cfg5.log; exit 9; }
tail -1 gpurun_out/base_cfg5.log
timeout -k 10 200 python -u bench.py --workload cfg4 --steps 5 --warmup 1 --no-side-configs --no-cpu-baseline > gpurun_out/base_cfg4.log 2>&1 || { echo cfg4 failed; exit 9; }
tail -1 gpurun_out/base_cfg4.log
