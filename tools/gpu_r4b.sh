#!/bin/bash
# Round 4: cooperative-launch stream-order check, GPU test suite, cold-path phases,
# then (only if cooperative launches were shown to skip the stream order and plain
# launches were not) the PM 1 cluster repro with the plain-launch library.
mkdir -p gpurun_out
O=gpurun_out/r4_coop.log
: > $O
timeout -k 10 120 ./tools/coop_order 300 1 >> $O 2>&1; r1=$?; echo "coop=1 rc=$r1" >> $O
[ $r1 -ge 2 ] && exit $r1
timeout -k 10 120 ./tools/coop_order 300 0 >> $O 2>&1; r0=$?; echo "coop=0 rc=$r0" >> $O
[ $r0 -ge 2 ] && exit $r0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r4_gputests.log 2>&1 || exit $?
timeout -k 10 180 python -u tools/cold_phases.py > gpurun_out/r4_cold.log 2>&1 || exit $?
if [ $r1 -eq 1 ] && [ $r0 -eq 0 ]; then
  REPS=6 timeout -k 10 240 python -u tools/repro_pm1.py "SHDR_CLUSTER_PM1=1" "SHDR_CLUSTER_PM1=1 SHDR_VARIANT=6" > gpurun_out/r4_pm1_plain.log 2>&1 || exit $?
  SHDR_LIB_VARIANT=verify REPS=3 timeout -k 10 240 python -u tools/repro_pm1.py "SHDR_CLUSTER_PM1=1" > gpurun_out/r4_pm1_plain_verify.log 2>&1 || exit $?
fi
