#!/bin/bash
# Round 4 session B: the 4-band SwinIR / SRRS validation diagnostics, the tap-row wgrad microbench,
# then A/B of the round-4 kernels inside one GPU call (box-to-box variance ~3 %):
# SwinIR fused attention half (SR_SWIN_FUSED=0 = three launches), ring wgrad row groups
# (SR_RING_VB=1 = 4-wave blocks) on RRDB, the tap-row wgrad on EDSR (SR_WG_TW=1), two co groups
# per ring-wgrad block on RCAN (SR_RING_CS=1; parity first)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_swin_fused_gpu.py \
  > $OUT/fused.log 2>&1; rc=$?; grep -E "fused|passed|failed|Error" $OUT/fused.log | cut -c1-300 | tail -12; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest -v -s --timeout 240 --timeout-method thread tests/test_srrs_model_gpu.py -k "four_band or validation" \
  > $OUT/srrs.log 2>&1; grep -E "4-band|validation psnr|passed|failed" $OUT/srrs.log | cut -c1-300
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_conv_gpu.py -k "wgrad_halo" \
  > $OUT/halo.log 2>&1; rc=$?; tail -3 $OUT/halo.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_conv.py 32 0,70,71,72 "256,256,64,0" > $OUT/bench_tw.log 2>&1 && grep wgrad $OUT/bench_tw.log || exit 1
ab() {  # $1 workload, $2 tag, rest: env
  wl=$1; tag=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/${wl}_$tag.log 2>&1 || { tail -20 $OUT/${wl}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${wl}_$tag.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.readline()); r=d['roofline'] or {}; k=r.get('kernels',{})
top=sorted(k.items(), key=lambda kv:-kv[1]['ms_per_step'])[:5]
print('$wl $tag', d['ms_per_step'], r.get('kernel'), r.get('frac'), [(n[:30], v['avg_us'], v['ms_per_step'], v.get('tflops')) for n,v in top])"
}
ab rcan cs SR_RING_CS=1 && ab rcan vb1 X=1 && ab rcan cs2 SR_RING_CS=1 && ab rcan vb1b X=1 && \
ab swinir fused X=1 && ab swinir unfused SR_SWIN_FUSED=0 && ab swinir fused2 X=1 && ab swinir unfused2 SR_SWIN_FUSED=0 && \
ab edsr tw SR_WG_TW=1 && ab edsr pp X=1 && ab rrdb vb2 X=1 && ab rrdb vb1 SR_RING_VB=1
