#!/bin/bash
# SwinIR step mode A/B: eager + side-stream weight gradients (default) vs HIP-graph replay, twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4sg
mkdir -p $OUT
for tag in eager graph eager2 graph2; do
  G=$([ "${tag#graph}" != "$tag" ] && echo 1 || echo -1)
  timeout -k 10 300 python -u bench.py --workload swinir --steps 20 --warmup 5 --no-cpu-baseline --no-parity --graph $G \
    > $OUT/swinir_$tag.log 2>&1 || { tail -20 $OUT/swinir_$tag.log; exit 1; }
  grep '^{"metric' $OUT/swinir_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('swinir $tag', d['ms_per_step'], d['config'].get('hip_graph'), d['config'].get('async_wgrad'))"
done
