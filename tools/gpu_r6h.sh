#!/bin/bash
# round 6: the 5x5 convolutions' stages by LDS-DMA (option conv_dma): equivalence test, one-box A/B
# of the C4 step, and the DMA form's PMC counters
mkdir -p gpurun_out/r6h
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -k "dma or fused_dgrad or conv_forward" -v --timeout 200 --timeout-method thread > gpurun_out/r6h/enc_tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_option.py conv_dma 0,1 --rounds 3 --steps 20 --config c4 > gpurun_out/r6h/ab_conv_dma.txt 2>&1 || exit 1
