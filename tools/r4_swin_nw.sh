#!/bin/bash
# SwinIR after the round's step changes: one-window attention blocks (SR_SWIN_ATTN_NW=1) vs two, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4swnw
mkdir -p $OUT
ab() {  # $1 tag, rest: env
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload swinir --steps 30 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/swinir_$tag.log 2>&1 || { tail -20 $OUT/swinir_$tag.log; return 1; }
  grep '^{"metric' $OUT/swinir_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('swinir $tag', d['ms_per_step'])"
}
ab nw2 X=1 && ab nw1 SR_SWIN_ATTN_NW=1 && ab nw2b X=1 && ab nw1b SR_SWIN_ATTN_NW=1
