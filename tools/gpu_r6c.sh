#!/bin/bash
# round 6: A/B of the top pair's factored weight-gradient role and of -fno-slp-vectorize against the
# default build (M step, eager, 200 steps, alternating order), and the factored form's metric-size
# parity
mkdir -p gpurun_out/r6c
L=$(pwd)/siren_mri_amd
SIREN_MRI_AMD_LIB=$L/libsiren_mri_amd_topfact.so timeout -k 10 300 python -u -m pytest tests/test_gpu_metric_parity.py -k "metric_size_forward_and_every_gradient or fused_loss" -v --timeout 200 --timeout-method thread > gpurun_out/r6c/topfact_parity.txt 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_libs.sh 3 $L/libsiren_mri_amd.so $L/libsiren_mri_amd_topfact.so $L/libsiren_mri_amd_noslp.so > gpurun_out/r6c/ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -k "four_wave or fused_dgrad or fused_node" -v --timeout 200 --timeout-method thread > gpurun_out/r6c/enc_tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c4 --no-psnr --no-cpu-baseline > gpurun_out/r6c/c4.json 2> gpurun_out/r6c/c4.err || exit 1
bash tools/prof_config.sh r6c/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline || exit 1
