#!/bin/bash
# where the pair kernels spend their cycles at the metric size and at the 1/8 shard
mkdir -p gpurun_out/r5i
export SIREN_MRI_AMD_LIB=$(pwd)/siren_mri_amd/libsiren_mri_amd_rprof.so
timeout -k 10 200 python tools/ring_profile.py --config m > gpurun_out/r5i/ring_m.txt 2>&1 || exit 1
timeout -k 10 200 python tools/ring_profile.py --config m_shard8 > gpurun_out/r5i/ring_sh8.txt 2>&1
