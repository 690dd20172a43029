set -e
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for roles in 2 1; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d "$R/gpurun_out/pp${roles}_pmc1" -o run --output-format csv -- python "$R/tools/pair_run.py" $roles 5 > "$R/gpurun_out/pp${roles}_pmc1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA -d "$R/gpurun_out/pp${roles}_pmc2" -o run --output-format csv -- python "$R/tools/pair_run.py" $roles 5 > "$R/gpurun_out/pp${roles}_pmc2.log" 2>&1
done
