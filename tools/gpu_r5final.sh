#!/bin/bash
# end of round 5: the new paths' tests, the whole GPU suite, smoke, the default bench line, the
# headline kernel profile and the C4 step profile
mkdir -p gpurun_out/r5f
timeout -k 10 600 python -u -m pytest tests/test_gpu_hyper.py tests/test_gpu_encoder.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5f/tests_new.txt 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5f/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f/smoke.txt 2>&1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/r5f/bench.json 2> gpurun_out/r5f/bench.err || exit 1
bash tools/prof_config.sh r5f/m --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-other-configs || exit 1
timeout -k 10 300 python bench.py --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline > gpurun_out/r5f/c4.json 2> gpurun_out/r5f/c4.err || exit 1
bash tools/prof_config.sh r5f/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline
