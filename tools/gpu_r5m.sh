#!/bin/bash
# fp64 stack parity
mkdir -p gpurun_out/r5m
timeout -k 10 400 python -u -m pytest tests/test_gpu_f64.py -v -s --timeout 120 --timeout-method thread > gpurun_out/r5m/f64.log 2>&1
