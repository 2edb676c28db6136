#!/bin/bash
# Round 4 session A: new-kernel parity (fused SwinIR attention half, two-row-group ring wgrad),
# workload tiles with their printed error maxima, real-image and SRRS-validation tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4a
mkdir -p $OUT
run_t() {  # $1 tag, rest: pytest args
  tag=$1; shift
  timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread "$@" > $OUT/$tag.log 2>&1
  rc=$?
  grep -E "passed|failed|error" $OUT/$tag.log | tail -2
  return $rc
}

run_t tw tests/test_conv_gpu.py -k "wgrad_tw or prepared_images" && \
run_t ring tests/test_conv_gpu.py -k "halo_vs_fp64 or ring" && \
run_t tiles tests/test_workload_tiles_gpu.py && \
run_t real tests/test_real_image_gpu.py tests/test_srrs_model_gpu.py && \
grep -h "bf16 B\|on baboon\|fused-unfused\|validation psnr" $OUT/*.log | cut -c1-330
timeout -k 10 300 python -u tools/bench_conv.py 32 0,70,71,72 "256,256,64,0" > $OUT/bench_tw.log 2>&1 && grep wgrad $OUT/bench_tw.log
