set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/exp.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 9; }
grep '^{' gpurun_out/bench.log | cut -c1-300
