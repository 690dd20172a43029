#!/bin/bash
# round 6: A/B of the top pair's factored weight-gradient role and of -fno-slp-vectorize against the
# default build (M step, eager, 200 steps, alternating order), and the factored form's metric-size
# parity
mkdir -p gpurun_out/r6c
L=$(pwd)/siren_mri_amd
SIREN_MRI_AMD_LIB=$L/libsiren_mri_amd_topfact.so timeout -k 10 300 python -u -m pytest tests/test_gpu_metric_parity.py -k "metric_size_forward_and_every_gradient or fused_loss" -v --timeout 200 --timeout-method thread > gpurun_out/r6c/topfact_parity.txt 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_libs.sh 3 $L/libsiren_mri_amd.so $L/libsiren_mri_amd_topfact.so $L/libsiren_mri_amd_noslp.so > gpurun_out/r6c/ab.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4_precision.py -v -s --timeout 880 --timeout-method thread > gpurun_out/r6c/c4_precision.txt 2>&1
timeout -k 10 400 python bench.py --config c4_fp32 --no-psnr --no-cpu-baseline > gpurun_out/r6c/c4_fp32.json 2> gpurun_out/r6c/c4_fp32.err || exit 1
