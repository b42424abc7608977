R="timeout -k 10 200 python -u tools/repro_cl.py"
SHDR_LIB_VARIANT=dbga $R "SHDR_CLUSTER=2" "SHDR_CLUSTER=4" > gpurun_out/repro_cl_a.log 2>&1
SHDR_LIB_VARIANT=dbgb $R "SHDR_CLUSTER=2" "SHDR_CLUSTER=4" > gpurun_out/repro_cl_b.log 2>&1
grep -h "rep\|shdr" gpurun_out/repro_cl_a.log gpurun_out/repro_cl_b.log
