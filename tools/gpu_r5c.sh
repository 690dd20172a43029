#!/bin/bash
# round-5 batch: FF exactness tests, C4 fused-input on/off, forward decomposition, r3-vs-HEAD A/B
mkdir -p gpurun_out/r5c
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_fourier_input.py \
  tests/test_gpu_wide.py::test_fourier_features_native_vs_reference tests/test_gpu_fused_loss.py "tests/test_gpu_metric_parity.py::test_metric_size_fp32_fused_loss_step_vs_oracle" > gpurun_out/r5c/ff.txt 2>&1 || echo "ff tests rc=$?"
for v in 0 1 4 8 64 128; do echo "== dbg $v"; timeout -k 5 60 build/fwd_f0_d$v 200 || exit 1; done > gpurun_out/r5c/fwd_dbg.txt 2>&1
SIREN_MRI_AMD_FUSED_FOURIER=0 timeout -k 10 200 python bench.py --config c4 --no-psnr --no-cpu-baseline > gpurun_out/r5c/c4_off.json 2> gpurun_out/r5c/c4_off.err || exit 1
SIREN_MRI_AMD_FUSED_FOURIER=1 timeout -k 10 200 python bench.py --config c4 --no-psnr --no-cpu-baseline > gpurun_out/r5c/c4_on.json 2> gpurun_out/r5c/c4_on.err || exit 1
bash tools/ab_tree.sh r5c/ab build/r3copy 2 > /dev/null 2>&1 || exit 1
