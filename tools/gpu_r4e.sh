#!/bin/bash
# Round 4: GPU suite (PM 1 clusters enabled), PM 1 cluster repro x6 per bucket width,
# cfg5 start-up phases, default bench line. Stops at the first failing step.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r4e_gputests.log 2>&1 || exit $?
REPS=6 timeout -k 10 300 python -u tools/repro_pm1.py "" "SHDR_VARIANT=6" > gpurun_out/r4e_pm1.log 2>&1 || exit $?
timeout -k 10 180 python -u tools/cold_phases.py > gpurun_out/r4e_cold.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r4e_bench.log 2>&1 || exit $?
