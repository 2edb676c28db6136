#!/bin/bash
# A/B of a Python-side switch inside ONE GPU call: runs bench.py with and without ENVVAR set.
# usage (GPU box): ENVVAR=SR_AB_UNFUSED WORKLOADS="rrdb" ROUNDS=2 bash tools/ab_env.sh
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in ${WORKLOADS:-edsr}; do
  for r in $(seq ${ROUNDS:-2}); do
    for v in off on; do
      if [ $v = on ]; then export $ENVVAR=1; else unset $ENVVAR; fi
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-trace --workload $w --steps ${STEPS:-10} --warmup 3 \
        > gpurun_out/abenv_${w}_$v.log 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/abenv_${w}_$v.log').read().strip().splitlines()[-1]); print('$w $ENVVAR=$v', d['ms_per_step'])"
    done
  done
done
