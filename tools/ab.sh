#!/bin/bash
# A/B of two builds of libsr_hip.so inside ONE GPU call (box-to-box variance is ~3 %):
# alternates bench.py runs of tools/ab/libA.so and tools/ab/libB.so.
# usage (GPU box): WORKLOADS="rcan rrdb" ROUNDS=2 bash tools/ab.sh
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in ${WORKLOADS:-edsr}; do
  for r in $(seq ${ROUNDS:-2}); do
    for v in A B; do
      SR_HIP_LIB=${ABDIR:-tools/ab}/lib$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-trace --workload $w \
        --steps ${STEPS:-10} --warmup 3 > gpurun_out/ab_${w}_$v.log 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/ab_${w}_$v.log').read().strip().splitlines()[-1]); print('$w $v', d['ms_per_step'])"
    done
  done
done
