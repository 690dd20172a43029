#!/bin/bash
# conv_fwd_k5 form 3 (the next stage's DMA issued one instruction per K step): encoder tests, A/B
mkdir -p gpurun_out/r6n
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6n/enc_tests.txt 2>&1 || { tail -30 gpurun_out/r6n/enc_tests.txt; exit 1; }
timeout -k 10 400 python -u tools/ab_option.py conv_dma 2,3,2,3 --rounds 2 --steps 60 --config c4 > gpurun_out/r6n/ab.txt 2>&1 || exit 1
tail -3 gpurun_out/r6n/enc_tests.txt; cat gpurun_out/r6n/ab.txt
