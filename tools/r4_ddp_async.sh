#!/bin/bash
# Round 4: why is the two-rank segmented-graph RCAN step with side-stream weight gradients 60x slower?
# Two gloo ranks on the one GPU; host timestamps per segment replay / all-reduce issue / join
# (SR_STEP_TRACE=host), then the same after a device sync per phase (SR_STEP_TRACE=sync).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4_ddp
mkdir -p $OUT
WL=${WL:-rcan}
run() {  # $1 tag, rest: env
  tag=$1; shift
  env "$@" SR_DIST_BACKEND=gloo timeout -k 10 240 python -u bench.py --gpus 2 --steps 3 --warmup 3 --workload $WL \
    --no-trace $EXTRA > $OUT/${WL}_$tag.log 2>&1 || { tail -30 $OUT/${WL}_$tag.log; return 1; }
  grep "^{\"metric" $OUT/${WL}_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$tag', d['ms_per_step'], d['config']['hip_graph'], d['config']['async_wgrad'])"
  grep step_trace $OUT/${WL}_$tag.log | tail -2
}
run sync_host SR_ASYNC_WGRAD=0 SR_STEP_TRACE=host || exit 1
run async_host SR_ASYNC_WGRAD=1 SR_STEP_TRACE=host || exit 1
run async_sync SR_ASYNC_WGRAD=1 SR_STEP_TRACE=sync || exit 1
run sync_sync SR_ASYNC_WGRAD=0 SR_STEP_TRACE=sync || exit 1
EXTRA="--graph 0" run eager_async SR_ASYNC_WGRAD=1 || exit 1
