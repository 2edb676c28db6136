#!/bin/bash
# RRDB's replayed step with side-stream weight gradients forked once per RRDB vs single-stream, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4rrdb
mkdir -p $OUT
ab() {  # $1 workload, $2 tag, rest: env
  wl=$1; tag=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/${wl}_$tag.log 2>&1 || { tail -20 $OUT/${wl}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${wl}_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$wl $tag', d['ms_per_step'], d['config'].get('async_wgrad'))"
}
ab rrdb async SR_BENCH_ASYNC_RRDB=1 && ab rrdb single X=1 && ab rrdb async2 SR_BENCH_ASYNC_RRDB=1 && ab rrdb single2 X=1
