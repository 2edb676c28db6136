#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gloo2
run() {  # $1 tag, rest: env / args
  tag=$1; shift
  env "$@" SR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 3 --workload rcan --no-trace $EXTRA > gpurun_out/gloo2/rcan_$tag.log 2>&1 || { tail -5 gpurun_out/gloo2/rcan_$tag.log; return 1; }
  grep '^{' gpurun_out/gloo2/rcan_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$tag', d['ms_per_step'], d['config']['hip_graph'], d['config']['async_wgrad'])"
}
run sync SR_ASYNC_WGRAD=0 || exit 1
EXTRA="--graph 0" run eager_sync SR_ASYNC_WGRAD=0 || exit 1
run default X=1 || exit 1
