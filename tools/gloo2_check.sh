#!/bin/bash
# two-rank gloo rehearsal of bench.py's distributed path (segmented graphs, bucketed reducer) on the one GPU
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gloo2
for w in ${WORKLOADS:-edsr rcan swinir rrdb}; do
  SR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 3 --workload $w > gpurun_out/gloo2/$w.log 2>&1 || { tail -20 gpurun_out/gloo2/$w.log; exit 1; }
  grep '^{' gpurun_out/gloo2/$w.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$w', d['n_gpus'], d['config']['parallelism'], d['ms_per_step'], d['last_loss'], d['config']['hip_graph'], d['config']['async_wgrad'])"
done
