#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_swin_ops_gpu.py tests/test_archs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lin or 1x1 or swin or Swin" > gpurun_out/lin_tests.log 2>&1
timeout -k 10 120 python3 tools/bench_conv.py 32 0 "184,552,64,0,1;184,368,64,0,1;184,184,64,0,1" > gpurun_out/lin_time.log 2>&1
WORKLOADS="swinir" bash tools/bench_all.sh
