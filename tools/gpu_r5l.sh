#!/bin/bash
# generic encoder convolutions: GPU encoder tests, then the C4 step's kernel profile
set -o pipefail
mkdir -p gpurun_out/r5l
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py -v --timeout 120 --timeout-method thread > gpurun_out/r5l/enc.log 2>&1
timeout -k 10 300 python bench.py --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline > gpurun_out/r5l/c4.json 2> gpurun_out/r5l/c4.err || exit 1
bash tools/prof_config.sh r5l/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline
