#!/bin/bash
# conv_wrw_k5 LDS-DMA form (option wrw_dma): encoder tests, then a one-box A/B on the C4 step
mkdir -p gpurun_out/r6j
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6j/enc_tests.txt 2>&1 || { tail -30 gpurun_out/r6j/enc_tests.txt; exit 1; }
timeout -k 10 400 python -u tools/ab_option.py wrw_dma 0,1,0,1 --rounds 3 --steps 60 --config c4 > gpurun_out/r6j/ab_wrw_dma.txt 2>&1 || exit 1
tail -3 gpurun_out/r6j/enc_tests.txt; cat gpurun_out/r6j/ab_wrw_dma.txt
