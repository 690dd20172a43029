#!/bin/bash
# native hypo_weight_loss: its test, the hypernetwork models' tests, the C4 step
mkdir -p gpurun_out/r5v
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper.py tests/test_gpu_modules.py tests/test_gpu_wide.py tests/test_gpu_fourier_input.py tests/test_gpu_fused_loss.py -v --timeout 300 --timeout-method thread > gpurun_out/r5v/tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline > gpurun_out/r5v/c4.json 2> gpurun_out/r5v/c4.err || exit 1
bash tools/prof_config.sh r5v/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline
