#!/bin/bash
# A/B of one library knob (environment variable) on a workload's bench step inside ONE GPU call.
# usage (GPU box): KNOB=SR_LN_BWD_RU VALS="1 4" WORKLOAD=swinir ROUNDS=2 bash tools/ab_knob.sh <tag>
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-abk}
mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for v in $VALS; do
    env $KNOB=$v timeout -k 10 300 python -u bench.py --workload ${WORKLOAD:-edsr} --no-cpu-baseline --no-parity --no-trace \
      --steps ${STEPS:-20} --warmup 5 > $OUT/${WORKLOAD}_${v}_r$r.json 2> $OUT/${WORKLOAD}_${v}_r$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/${WORKLOAD}_${v}_r$r.json').read().strip().splitlines()[-1]); print('${WORKLOAD} $KNOB=$v r$r', d['ms_per_step'])"
  done
done
