#!/bin/bash
# GPU box: eager (DDP-path) step time of RCAN / SwinIR with and without the side-stream weight
# gradients, and the two-rank gloo rehearsal of bench.py's distributed path on the one GPU.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in rcan swinir; do
  for v in 0 1; do
    SR_ASYNC_WGRAD=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity --no-trace --graph 0 --workload $w \
      --steps 6 --warmup 3 > gpurun_out/eager_${w}_$v.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/eager_${w}_$v.log').read().strip().splitlines()[-1]); print('$w eager async=$v', d['ms_per_step'])"
  done
done
SR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --workload rcan > gpurun_out/gloo2_rcan.log 2>&1 || exit 1
grep '^{' gpurun_out/gloo2_rcan.log | cut -c1-300
