# Scratch A/B: parity tests on the experiment flavour, then bench base vs flavour (cfg4 x2, cfg5 x1).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/exp.log
FL=${FL:-new}
SHDR_LIB_VARIANT=$FL timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit 1; }
run() { timeout -k 10 300 "$@" --no-cpu-baseline --no-side-configs > gpurun_out/one.json 2>>gpurun_out/exp.log || { echo "FATAL"; tail gpurun_out/exp.log; exit 9; }; python -c "import json;d=json.loads(open('gpurun_out/one.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],2),round(d['roofline']['kernel_ms'],2),d['roofline']['kernel_ms_each'])"; }
for i in 1 2; do
  echo -n "base: "; run python -u bench.py --steps 5
  echo -n "$FL: "; SHDR_LIB_VARIANT=$FL run python -u bench.py --steps 5
done
if [ -z "$NO_CFG5" ]; then
  echo -n "cfg5 base: "; run python -u bench.py --workload cfg5 --steps 1 --warmup 1
  echo -n "cfg5 $FL: "; SHDR_LIB_VARIANT=$FL run python -u bench.py --workload cfg5 --steps 1 --warmup 1
fi
