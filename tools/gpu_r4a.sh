#!/bin/bash
# Round 4: cooperative-launch stream-order check, then the GPU test suite.
mkdir -p gpurun_out
O=gpurun_out/r4_coop.log
: > $O
for c in 1 0; do
  timeout -k 10 120 ./tools/coop_order 300 $c >> $O 2>&1; rc=$?
  echo "coop=$c rc=$rc" >> $O
  [ $rc -ge 2 ] && exit $rc
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r4_gputests.log 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -u tools/cold_phases.py > gpurun_out/r4_cold.log 2>&1
