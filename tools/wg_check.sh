#!/bin/bash
# ring wgrad: correctness, then timing vs the tile-row halo form (variant 37)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/wg_tests.log 2>&1
timeout -k 10 300 python -u tools/bench_conv.py 32 0,37 "64,64,64,0" > gpurun_out/wg_bench.log 2>&1
timeout -k 10 300 python -u tools/bench_conv.py 16 0,37 "64,32,128,0;192,64,128,0;32,64,128,0" >> gpurun_out/wg_bench.log 2>&1
bash tools/wg_prof.sh > /dev/null
