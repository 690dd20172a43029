#!/bin/bash
# grouped native hypernet heads: parity, the C4 callers' tests, the C4 step profile
mkdir -p gpurun_out/r5r
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper.py tests/test_gpu_encoder.py tests/test_gpu_modules.py tests/test_gpu_wide.py tests/test_gpu_fourier_input.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5r/tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline > gpurun_out/r5r/c4.json 2> gpurun_out/r5r/c4.err || exit 1
bash tools/prof_config.sh r5r/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline
