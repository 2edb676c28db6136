#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
# 35: 64 blocks (full); 36+1=37: 64 blocks no MFMA; 38: 64 blocks no epilogue; 39: neither
timeout -k 10 300 python -u tools/bench_conv.py 32 0,34,35,37,38,39 "64,64,64,0" > gpurun_out/band_ablate.log 2>&1
