#!/bin/bash
# Round 4 session B: A/B of the round-4 kernels inside one GPU call (box-to-box variance ~3 %):
# SwinIR fused attention half (SR_SWIN_FUSED=0 = three launches), ring wgrad row groups
# (SR_RING_VB=1 = 4-wave blocks) on RRDB and RCAN
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4b
mkdir -p $OUT
ab() {  # $1 workload, $2 tag, rest: env
  wl=$1; tag=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/${wl}_$tag.log 2>&1 || { tail -20 $OUT/${wl}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${wl}_$tag.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.readline()); r=d['roofline'] or {}; k=r.get('kernels',{})
top=sorted(k.items(), key=lambda kv:-kv[1]['ms_per_step'])[:4]
print('$wl $tag', d['ms_per_step'], r.get('kernel'), r.get('frac'), [(n[:28], v['avg_us'], v['ms_per_step']) for n,v in top])"
}
ab swinir fused X=1 && ab swinir unfused SR_SWIN_FUSED=0 && ab swinir fused2 X=1 && ab swinir unfused2 SR_SWIN_FUSED=0 && \
ab rrdb vb2 X=1 && ab rrdb vb1 SR_RING_VB=1 && ab rrdb vb2b X=1 && ab rrdb vb1b SR_RING_VB=1 && \
ab rcan vb2 X=1 && ab edsr base X=1
