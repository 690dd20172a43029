#!/bin/bash
# PMC counters of the forward kernel for library variants (one counter pass per run):
#   bash tools/pmc_probe.sh TAG name1 name2 ...   -> gpurun_out/TAG_<name>_pmc*/, summary on stdout
set -e
TAG=$1; shift
R=$(pwd)
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for n in "$@"; do
  if [ "$n" = base ]; then lib=$R/siren_mri_amd/libsiren_mri_amd.so; else lib=$R/siren_mri_amd/libsiren_mri_amd_$n.so; fi
  export SIREN_MRI_AMD_LIB=$lib
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES \
      -d "$R/gpurun_out/${TAG}_${n}_pmc1" -o run --output-format csv -- python "$R/tools/freg_probe.py" 0 > "$R/gpurun_out/${TAG}_${n}_pmc1.log" 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS \
      SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT \
      -d "$R/gpurun_out/${TAG}_${n}_pmc2" -o run --output-format csv -- python "$R/tools/freg_probe.py" 0 > "$R/gpurun_out/${TAG}_${n}_pmc2.log" 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE \
      -d "$R/gpurun_out/${TAG}_${n}_pmc3" -o run --output-format csv -- python "$R/tools/freg_probe.py" 0 > "$R/gpurun_out/${TAG}_${n}_pmc3.log" 2>&1
done
cd "$R"
python tools/pmc_kernel_summary.py "gpurun_out/${TAG}" fused_fwd_reg "$@"
