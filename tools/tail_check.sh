#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "tail" > gpurun_out/tail_tests.log 2>&1
timeout -k 10 120 python3 tools/bench_conv.py 32 0,29 "256,3,256,0" > gpurun_out/tail_time.log 2>&1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_edsr_tail.log 2>&1
