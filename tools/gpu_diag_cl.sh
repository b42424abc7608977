set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_cluster.sh tests || exit 1
for c in 1 2 3; do
  SHDR_CLUSTER=$c PART=8 timeout -k 10 120 python -u tools/diag.py 4 cfg4 > gpurun_out/diag_cl$c.log 2>&1 || exit 1
done
for c in 1 2; do
  SHDR_CLUSTER=$c PART=8 timeout -k 10 200 python -u tools/diag.py 4 cfg5 > gpurun_out/diag5_cl$c.log 2>&1 || exit 1
done
env REPS=2 PART=8 PARTS_MAX=3 timeout -k 10 300 python -u tools/ab.py cfg4 "" "SHDR_CLUSTER=2" "SHDR_CLUSTER=3" "SHDR_CLUSTER=4 SHDR_VARIANT=7" > gpurun_out/cl_ab_cfg4.log 2>&1 || exit 2
tail -5 gpurun_out/cl_ab_cfg4.log
