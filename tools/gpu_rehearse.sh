#!/bin/bash
# Multi-rank bench rehearsal on ONE GPU: 2 ranks (gloo backend, both on cuda:0), strong scaling
# over the coherent partition, the table all-gather and the MIN all-reduce. Not a scaling number.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --workload ${W:-cfg4} --backend gloo --same-device \
  > gpurun_out/rehearse.log 2>&1 || { echo rehearsal failed; tail -30 gpurun_out/rehearse.log; exit 9; }
grep '^{"metric"' gpurun_out/rehearse.log | tail -1
