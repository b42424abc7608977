set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -25 gpurun_out/gpu_tests.log
case $rc in 0|1) ;; *) echo "FATAL tests rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_cfg4.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_cfg4.log; exit 9; }
tail -3 gpurun_out/bench_cfg4.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ktrace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/prof_ktrace.log 2>&1 || { echo prof failed; tail -30 gpurun_out/prof_ktrace.log; exit 9; }
find gpurun_out/prof_ktrace -name '*stats*'
