#!/bin/bash
# conv_fwd_k5 stage-fill form 2 (per-workgroup DMA offsets): encoder tests, then a one-box A/B
# of option conv_dma 1 vs 2 on the C4 step
mkdir -p gpurun_out/r6i
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6i/enc_tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_option.py conv_dma 1,2,1,2 --rounds 3 --steps 60 --config c4 > gpurun_out/r6i/ab_conv_dma2.txt 2>&1 || exit 1
tail -3 gpurun_out/r6i/enc_tests.txt; cat gpurun_out/r6i/ab_conv_dma2.txt
