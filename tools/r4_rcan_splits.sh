#!/bin/bash
# RCAN after the batched forks: ring-wgrad split target (SR_RING_SPLITS) 512 (default) vs 256 / 1024, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4rcs
mkdir -p $OUT
ab() {  # $1 tag, rest: env
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload rcan --steps 30 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/rcan_$tag.log 2>&1 || { tail -20 $OUT/rcan_$tag.log; return 1; }
  grep '^{"metric' $OUT/rcan_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('rcan $tag', d['ms_per_step'])"
}
ab s512 X=1 && ab s256 SR_RING_SPLITS=256 && ab s1024 SR_RING_SPLITS=1024 && ab s512b X=1 && ab s256b SR_RING_SPLITS=256 && \
  ab s1024b SR_RING_SPLITS=1024
