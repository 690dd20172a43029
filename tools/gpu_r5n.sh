#!/bin/bash
# A/B: dw-role slab written as coalesced 16-byte stores in fragment order (timing probe) vs the
# row-major dword stores
mkdir -p gpurun_out/r5n
R=$(pwd)
for v in base fragp base2 fragp2; do
  if [ "${v%2}" = fragp ]; then export SIREN_MRI_AMD_LIB=$R/siren_mri_amd/libsiren_mri_amd_fragp.so; else unset SIREN_MRI_AMD_LIB; fi
  bash tools/prof_config.sh r5n/sh8_$v --config m_shard8 --steps 50 --warmup 10 --no-psnr --no-cpu-baseline --no-other-configs || exit 1
done
