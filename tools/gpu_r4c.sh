#!/bin/bash
# Round 4: GPU suite, default bench line, then the PM 1 cluster repro (verify flavour
# first: relaxation postconditions + poisoned predecessors; then the product).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r4c_gputests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r4c_bench.log 2>&1 || exit $?
SHDR_LIB_VARIANT=verify REPS=3 timeout -k 10 240 python -u tools/repro_pm1.py "" "SHDR_VARIANT=6" > gpurun_out/r4c_pm1_verify.log 2>&1 || exit $?
REPS=4 timeout -k 10 240 python -u tools/repro_pm1.py "" "SHDR_VARIANT=6" > gpurun_out/r4c_pm1_prod.log 2>&1 || exit $?
