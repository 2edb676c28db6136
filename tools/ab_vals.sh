#!/bin/bash
# A/B of an environment knob over several values inside ONE GPU call (bench.py step time).
# usage (GPU box): VAR=SR_RING_SPLITS VALUES="128 512" WL=rcan ROUNDS=2 bash tools/ab_vals.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abv
for r in $(seq ${ROUNDS:-2}); do
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-trace --workload ${WL:-edsr} \
      --steps ${STEPS:-10} --warmup 3 > gpurun_out/abv/${WL:-edsr}_${VAR}_${v}_$r.log 2>&1 \
      || { tail -20 gpurun_out/abv/${WL:-edsr}_${VAR}_${v}_$r.log; exit 2; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abv/${WL:-edsr}_${VAR}_${v}_$r.log').read().strip().splitlines()[-1]); print('${WL:-edsr} $VAR=$v', d['ms_per_step'], d.get('last_loss'))"
  done
done
