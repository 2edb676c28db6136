#!/bin/bash
# GPU box: SR_ASYNC_WGRAD=0 / reduce / 1 on one workload (ROUNDS alternations)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in ${WORKLOADS:-edsr}; do
  for r in $(seq ${ROUNDS:-2}); do
    for v in 0 reduce; do
      SR_ASYNC_WGRAD=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-trace --no-parity --workload $w \
        --steps ${STEPS:-10} --warmup 3 > gpurun_out/abenv3_${w}_$v.log 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/abenv3_${w}_$v.log').read().strip().splitlines()[-1]); print('$w async=$v', d['ms_per_step'])"
    done
  done
done
