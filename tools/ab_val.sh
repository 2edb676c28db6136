#!/bin/bash
# Sweep of an environment knob inside ONE GPU call: bench.py once per VALUE (and ROUNDS times).
# usage (GPU box): VAR=SR_RING_SPLITS VALUES="512 256 128" WORKLOADS="rcan" ROUNDS=2 bash tools/ab_val.sh
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in ${WORKLOADS:-edsr}; do
  for r in $(seq ${ROUNDS:-2}); do
    for v in $VALUES; do
      export $VAR=$v
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-trace --no-parity --workload $w --steps ${STEPS:-10} \
        --warmup 3 > gpurun_out/abval_${w}_$v.log 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/abval_${w}_$v.log').read().strip().splitlines()[-1]); print('$w $VAR=$v', d['ms_per_step'])"
    done
  done
done
