#!/bin/bash
# EDSR's replayed step with side-stream weight gradients (one fork per 4 / 8 / 16 ResBlocks)
# vs single-stream, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4edsr
mkdir -p $OUT
ab() {  # $1 workload, $2 tag, rest: env
  wl=$1; tag=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/${wl}_$tag.log 2>&1 || { tail -20 $OUT/${wl}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${wl}_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$wl $tag', d['ms_per_step'], d['config'].get('async_wgrad'))"
}
ab edsr single X=1 && ab edsr k4 SR_BENCH_ASYNC=edsr && ab edsr k8 SR_BENCH_ASYNC=edsr SR_SIDE_BATCH=8 && \
  ab edsr k16 SR_BENCH_ASYNC=edsr SR_SIDE_BATCH=16 && ab edsr single2 X=1 && ab edsr k4b SR_BENCH_ASYNC=edsr && \
  ab edsr k8b SR_BENCH_ASYNC=edsr SR_SIDE_BATCH=8 && ab edsr k16b SR_BENCH_ASYNC=edsr SR_SIDE_BATCH=16 && \
  ab edsr single3 X=1 && ab edsr k4c SR_BENCH_ASYNC=edsr && ab edsr k8c SR_BENCH_ASYNC=edsr SR_SIDE_BATCH=8
