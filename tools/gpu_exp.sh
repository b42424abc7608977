set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/exp.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --same-device --steps 2 --warmup 1 > gpurun_out/bench_rehearsal2.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_rehearsal2.log | cut -c1-600; [ $rc -eq 0 ] || { echo "rehearsal failed rc=$rc"; tail -20 gpurun_out/bench_rehearsal2.log; exit 1; }
timeout -k 10 400 python -u bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg5.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_cfg5.log | cut -c1-900; [ $rc -eq 0 ] || { echo "cfg5 failed rc=$rc"; tail -20 gpurun_out/bench_cfg5.log; exit 1; }
