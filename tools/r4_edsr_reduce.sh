#!/bin/bash
# EDSR with only the split-K slab reduces on the side stream (SR_ASYNC_WGRAD=reduce, forked once per
# ResBlock through side_batch) vs single-stream, alternating; the async bitwise tests first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4edsr_red
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_train_step_gpu.py \
  -k "async" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log | cut -c1-200; [ $rc -eq 0 ] || exit 1
ab() {  # $1 tag, rest: env
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload edsr --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/edsr_$tag.log 2>&1 || { tail -20 $OUT/edsr_$tag.log; return 1; }
  grep '^{"metric' $OUT/edsr_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('edsr $tag', d['ms_per_step'], d['config'].get('async_wgrad'))"
}
ab single X=1 && ab reduce SR_ASYNC_WGRAD=reduce && ab single2 X=1 && ab reduce2 SR_ASYNC_WGRAD=reduce && \
  ab single3 X=1 && ab reduce3 SR_ASYNC_WGRAD=reduce
