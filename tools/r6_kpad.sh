#!/bin/bash
# K-padded 184-channel conv forwards (SR_CONV_KPAD): the SwinIR step with / without, traced (the default
# bench line) and untraced, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-kpad}; mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for v in unset 0; do
    if [ $v = unset ]; then unset SR_CONV_KPAD; else export SR_CONV_KPAD=$v; fi
    timeout -k 10 300 python -u bench.py --workload swinir --no-cpu-baseline > $OUT/full_${v}_$r.log 2>&1 || exit 1
    timeout -k 10 300 python -u bench.py --workload swinir --no-cpu-baseline --no-trace --no-parity > $OUT/notrace_${v}_$r.log 2>&1 || exit 1
    python3 -c "
import json
f = lambda p: json.loads([l for l in open(p) if l.startswith('{\"metric')][-1])['ms_per_step']
print('round $r SR_CONV_KPAD=$v full', f('$OUT/full_${v}_$r.log'), 'notrace', f('$OUT/notrace_${v}_$r.log'))"
  done
done
