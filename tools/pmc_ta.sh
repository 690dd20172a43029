#!/bin/bash
# Texture-address / L1 counters of the forward kernel per library variant (one counter group per run):
#   bash tools/pmc_ta.sh TAG name1 name2 ...
R=$(pwd)
TAG=$1; shift
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for n in "$@"; do
  if [ "$n" = base ]; then lib=$R/siren_mri_amd/libsiren_mri_amd.so; else lib=$R/siren_mri_amd/libsiren_mri_amd_$n.so; fi
  export SIREN_MRI_AMD_LIB=$lib
  k=0
  for grp in "TA_BUSY_avr TA_BUFFER_TOTAL_CYCLES_sum GRBM_GUI_ACTIVE" \
             "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
             "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
             "TA_BUFFER_WRITE_WAVEFRONTS_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum"; do
    k=$((k + 1))
    timeout -s KILL 90 rocprofv3 --pmc $grp -d "$R/gpurun_out/${TAG}_${n}_pmc$k" -o run --output-format csv -- \
      python "$R/tools/freg_probe.py" 0 > "$R/gpurun_out/${TAG}_${n}_pmc$k.log" 2>&1 || echo "pass $k failed"
  done
done
cd "$R"
python tools/pmc_kernel_summary.py "gpurun_out/${TAG}" fused_fwd_reg "$@"
