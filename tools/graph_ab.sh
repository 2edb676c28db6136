#!/bin/bash
# GPU box: graph replay vs eager step (bench.py --graph 1 / 0) per workload, ROUNDS alternations
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in ${WORKLOADS:-swinir}; do
  for r in $(seq ${ROUNDS:-2}); do
    for gph in 1 0; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity --no-trace --graph $gph --workload $w \
        --steps ${STEPS:-8} --warmup 3 > gpurun_out/gab_${w}_$gph.log 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/gab_${w}_$gph.log').read().strip().splitlines()[-1]); print('$w graph=$gph', d['ms_per_step'])"
    done
  done
done
