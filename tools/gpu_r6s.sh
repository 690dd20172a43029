#!/bin/bash
# generic-shape weight gradient in 128-pixel LDS-DMA chunks (option wrw_dma 3): encoder tests, C4 A/B
mkdir -p gpurun_out/r6s
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6s/tests.txt 2>&1 || { tail -30 gpurun_out/r6s/tests.txt; exit 1; }
timeout -k 10 400 python -u tools/ab_option.py wrw_dma 2,3,2,3 --rounds 2 --steps 60 --config c4 > gpurun_out/r6s/ab.txt 2>&1 || exit 1
tail -2 gpurun_out/r6s/tests.txt; cat gpurun_out/r6s/ab.txt
