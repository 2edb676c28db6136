#!/bin/bash
# band kernel: correctness tests, then timing vs the tile kernel (variant 34), then phase stamps
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "band or halo or colsum" > gpurun_out/band_tests.log 2>&1
timeout -k 10 300 python -u tools/bench_conv.py 32 36,34,35 "64,64,64,0" > gpurun_out/band_bench.log 2>&1
timeout -k 10 300 python -u tools/band_stamps.py 32 36,35,37,38,39 64,64,64 > gpurun_out/band_stamps.log 2>&1
