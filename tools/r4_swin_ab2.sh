#!/bin/bash
# SwinIR after the batched side-stream forks: fused LayerNorm backward (SR_LN_BWD_FUSED=1) and graph
# replay (--graph 1) against the default eager step, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4swab2
mkdir -p $OUT
ab() {  # $1 tag, $2 graph flag, rest: env
  tag=$1; G=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload swinir --steps 30 --warmup 5 --no-cpu-baseline --no-parity \
    --graph $G > $OUT/swinir_$tag.log 2>&1 || { tail -20 $OUT/swinir_$tag.log; return 1; }
  grep '^{"metric' $OUT/swinir_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('swinir $tag', d['ms_per_step'])"
}
ab base -1 X=1 && ab lnb -1 SR_LN_BWD_FUSED=1 && ab graph 1 X=1 && ab graph_lnb 1 SR_LN_BWD_FUSED=1 && \
  ab base2 -1 X=1 && ab lnb2 -1 SR_LN_BWD_FUSED=1 && ab graph2 1 X=1 && ab graph_lnb2 1 SR_LN_BWD_FUSED=1
