#!/bin/bash
# round 6, first GPU call: the new tests (ADVICE r5 fixes, C4 bf16-vs-fp32 at equal steps), the C3
# kernel profile of the current state, and the default bench line
mkdir -p gpurun_out/r6a
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_hyper.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r6a/tests_new.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4_precision.py -v -s --timeout 500 --timeout-method thread > gpurun_out/r6a/c4_precision.txt 2>&1
timeout -k 10 300 python bench.py --config c3 --no-psnr --no-cpu-baseline > gpurun_out/r6a/c3.json 2> gpurun_out/r6a/c3.err || exit 1
bash tools/prof_config.sh r6a/c3 --config c3 --timing eager --steps 10 --warmup 3 --no-psnr --no-cpu-baseline || exit 1
timeout -k 10 300 python bench.py --config c4_fp32 --no-psnr --no-cpu-baseline > gpurun_out/r6a/c4_fp32.json 2> gpurun_out/r6a/c4_fp32.err || exit 1
timeout -k 10 500 python bench.py --no-cpu-baseline > gpurun_out/r6a/bench.json 2> gpurun_out/r6a/bench.err || exit 1
