#!/bin/bash
# 5x5 weight gradient in 128-pixel chunks (option wrw_dma 2): encoder tests, one-box A/B on C4
mkdir -p gpurun_out/r6m
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6m/enc_tests.txt 2>&1 || { tail -30 gpurun_out/r6m/enc_tests.txt; exit 1; }
timeout -k 10 400 python -u tools/ab_option.py wrw_dma 1,2,1,2 --rounds 2 --steps 60 --config c4 > gpurun_out/r6m/ab.txt 2>&1 || exit 1
tail -3 gpurun_out/r6m/enc_tests.txt; cat gpurun_out/r6m/ab.txt
