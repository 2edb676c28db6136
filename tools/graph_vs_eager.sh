#!/bin/bash
# GPU box: ms/step of each workload eager (the DDP path) vs HIP-graph replay.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in ${WORKLOADS:-edsr rcan swinir rrdb}; do
  for g in 0 1; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload $w --graph $g --steps ${STEPS:-10} --warmup 3 \
      > gpurun_out/ge_${w}_$g.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ge_${w}_$g.log').read().strip().splitlines()[-1]); print('$w graph=$g', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'])"
  done
done
