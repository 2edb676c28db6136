#!/bin/bash
# A/B of an environment knob over several values inside ONE GPU call (alternating rounds):
#   VAR=SR_RING_RED VALS="0 4" WORKLOADS="rcan rrdb" ROUNDS=2 bash tools/ab_vals.sh <tag>
# -> gpurun_out/<tag>/ab_<workload>_<val>_<round>.log, one summary line per run
TAG=${1:-ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
for w in ${WORKLOADS:-rcan}; do
  for r in $(seq ${ROUNDS:-2}); do
    for v in ${VALS:-0 1}; do
      if [ "$v" = unset ]; then unset $VAR; else export $VAR=$v; fi
      f=$OUT/ab_${w}_$(basename $v)_$r.log
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-trace --no-parity --workload $w --steps ${STEPS:-20} \
        --warmup 5 > $f 2>&1 || { tail -20 $f; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{\"metric')][-1]); print('$w $VAR=$v round $r', d['ms_per_step'])"
    done
  done
done
