#!/bin/bash
# K-padded 184-channel convs on the halo-row 256x256 kernel: tests, then the SwinIR step with / without
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-kpad}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_workload_tiles_gpu.py tests/test_swin_fused_gpu.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider -k "kpad or swinir or swin" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
VAR=SR_CONV_KPAD VALS="unset 0" WORKLOADS=swinir ROUNDS=${ROUNDS:-2} bash tools/ab_vals.sh ${1:-kpad}
