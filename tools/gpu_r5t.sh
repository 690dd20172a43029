#!/bin/bash
# advisor lows: first-order dx under create_graph, image gradient through the encoder
mkdir -p gpurun_out/r5t
timeout -k 10 600 python -u -m pytest tests/test_gpu_jvp.py tests/test_gpu_encoder.py tests/test_gpu_optim.py -v --timeout 300 --timeout-method thread > gpurun_out/r5t/tests.txt 2>&1
