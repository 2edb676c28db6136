#!/bin/bash
# EDSR's two ring weight gradients (conv_first 3 -> 256, conv_last 256 -> 3 at 256^2): split target
# (SR_RING_SPLITS) and ring depth (SR_RING_D) A/B on the EDSR step and the ring kernels' times; then
# the SwinIR host / GPU time per eager step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4edsr_ring
mkdir -p $OUT
ab() {  # $1 tag, rest: env
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload edsr --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/edsr_$tag.log 2>&1 || { tail -20 $OUT/edsr_$tag.log; return 1; }
  grep '^{"metric' $OUT/edsr_$tag.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.readline()); k=d['roofline']['kernels']
print('edsr $tag', d['ms_per_step'], [(n, v['avg_us'], v['calls']) for n, v in k.items() if 'ring' in n or 'tail' in n or 'pp_kernel' in n])"
}
ab base X=1 && ab s1024 SR_RING_SPLITS=1024 && ab s2048 SR_RING_SPLITS=2048 && ab d4 SR_RING_D=4 && ab base2 X=1 && \
  ab s1024b SR_RING_SPLITS=1024
timeout -k 10 200 python -u tools/replay_gap.py --workload swinir --steps 8
