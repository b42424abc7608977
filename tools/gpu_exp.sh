set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/exp.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
run() { echo "== $*"; timeout -k 10 200 "$@" >> gpurun_out/exp.log 2>&1; rc=$?; [ $rc -eq 0 ] || { echo "FATAL rc=$rc"; tail gpurun_out/exp.log; exit $rc; }; }
for d in 0 8 16 32 64 128; do echo "split_deg $d" >> gpurun_out/exp.log; SHDR_SPLIT_DEG=$d run python -u tools/exp.py cfg4 4; done
cat gpurun_out/exp.log | grep -v amdgpu.ids
