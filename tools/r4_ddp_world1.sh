#!/bin/bash
# Round 4: the distributed step (reducer + segmented HIP graphs + RCCL) at world 1, one process on
# the GPU, against the single-process graph step: does the segmented graph with side-stream weight
# gradients run as fast as the plain graph when each rank owns its GPU?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4_ddp1
mkdir -p $OUT
WL=${WL:-rcan}
run() {  # $1 tag, rest: bench args
  tag=$1; shift
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --workload $WL --no-cpu-baseline --no-parity --no-trace "$@" \
    > $OUT/${WL}_$tag.log 2>&1 || { tail -30 $OUT/${WL}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${WL}_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$tag', d['ms_per_step'], d['config']['parallelism'], d['config']['hip_graph'], d['config']['async_wgrad'])"
}
run graph_async || exit 1
run ddp_graph_async --ddp || exit 1
SR_ASYNC_WGRAD=0 run ddp_graph_sync --ddp || exit 1
SR_STEP_TRACE=host run ddp_graph_async_trace --ddp || exit 1
grep step_trace $OUT/${WL}_ddp_graph_async_trace.log | tail -1
WL=edsr run graph || exit 1
WL=edsr run ddp_graph --ddp || exit 1
