#!/bin/bash
# band kernel: correctness tests, then timing vs the tile kernel (variant 34)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "band or halo or colsum" > gpurun_out/band_tests.log 2>&1
timeout -k 10 300 python -u tools/bench_conv.py 32 36,34,35 "64,64,64,0" > gpurun_out/band_bench.log 2>&1
timeout -k 10 300 python -u tools/bench_conv.py 16 36,34 "64,32,128,0;32,64,128,0" >> gpurun_out/band_bench.log 2>&1
