#!/bin/bash
# Round 4 SwinIR session: parity of the fused block halves, then A/B fused vs unfused
# (SR_SWIN_FUSED=0) on the SwinIR-M bench, twice, in one GPU call (box-to-box variance ~3 %).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4swin
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_swin_fused_gpu.py \
  > $OUT/fused.log 2>&1; rc=$?; grep -E "fused|passed|failed|Error" $OUT/fused.log | cut -c1-300 | tail -12; [ $rc -eq 0 ] || exit 1
ab() {  # $1 workload, $2 tag, rest: env
  wl=$1; tag=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/${wl}_$tag.log 2>&1 || { tail -20 $OUT/${wl}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${wl}_$tag.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.readline()); r=d['roofline'] or {}; k=r.get('kernels',{})
top=sorted(k.items(), key=lambda kv:-kv[1]['ms_per_step'])[:7]
print('$wl $tag', d['ms_per_step'], r.get('kernel'), r.get('frac'), d.get('swin_fused_attention'), [(n[:30], v['avg_us'], v['ms_per_step'], v.get('tflops')) for n,v in top])"
}
ab swinir nw2 X=1 && ab swinir nw1 SR_SWIN_ATTN_NW=1 && ab swinir unfused SR_SWIN_FUSED=0 && ab swinir nw2b X=1 && \
  ab swinir nw1b SR_SWIN_ATTN_NW=1
