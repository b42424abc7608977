#!/bin/bash
# Multi-rank bench rehearsal on ONE GPU: 2 ranks (gloo backend, both on cuda:0), strong scaling
# over the coherent partition, the MIN all-reduce (and, for cfg4, the table all-gather). Not a
# scaling number: both ranks share one GPU (engines told so: no cluster mode).
set -o pipefail
mkdir -p gpurun_out
for w in cfg4 cfg5; do
  extra=""; [ $w = cfg5 ] && extra="--no-gather"
  SHDR_ENGINES_SHARE_DEVICES=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --workload $w --backend gloo --same-device $extra \
    > gpurun_out/rehearse_$w.log 2>&1 || { echo rehearsal $w failed; tail -30 gpurun_out/rehearse_$w.log; exit 9; }
  grep '^{"metric"' gpurun_out/rehearse_$w.log | tail -1
done
