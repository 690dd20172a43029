#!/bin/bash
# round 6: conflict-free staging writes in the encoder convolutions and the weight-gradient loader
# cursor: encoder tests, C4 bench, C4 kernel profile (summarised on the box), C4 PMC passes
mkdir -p gpurun_out/r6g
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -v --timeout 300 --timeout-method thread > gpurun_out/r6g/enc_tests.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c4 --no-psnr --no-cpu-baseline > gpurun_out/r6g/c4.json 2> gpurun_out/r6g/c4.err || exit 1
bash tools/prof_config.sh r6g/c4 --config c4 --timing eager --steps 5 --warmup 2 --no-psnr --no-cpu-baseline || exit 1
python tools/step_kernels.py gpurun_out/r6g/c4_prof/run_kernel_trace.csv 3 > gpurun_out/r6g/c4_step_kernels.txt
rm -f gpurun_out/r6g/c4_prof/run_kernel_trace.csv
bash tools/pmc_step.sh r6g/c4 --config c4 --timing eager > gpurun_out/r6g/c4_pmc.log 2>&1 || exit 1
find gpurun_out/r6g -name '*counter_collection.csv' -size +2M -delete
du -sh gpurun_out/r6g
