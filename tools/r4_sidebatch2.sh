#!/bin/bash
# Blocks per side-stream fork (SR_SIDE_BATCH=k): RCAN and SwinIR at k = 1, 2, 4, alternating; the
# async / DDP GPU tests at k = 4 first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4sb2
mkdir -p $OUT
SR_SIDE_BATCH=4 timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_train_step_gpu.py tests/test_ddp_gpu.py > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" $OUT/tests.log | cut -c1-300 | tail -8; [ $rc -eq 0 ] || exit 1
ab() {  # $1 workload, $2 tag, rest: env
  wl=$1; tag=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/${wl}_$tag.log 2>&1 || { tail -20 $OUT/${wl}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${wl}_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$wl $tag', d['ms_per_step'])"
}
ab rcan k1 SR_SIDE_BATCH=1 && ab rcan k2 SR_SIDE_BATCH=2 && ab rcan k4 SR_SIDE_BATCH=4 && ab rcan k20 SR_SIDE_BATCH=20 && \
  ab rcan k1b SR_SIDE_BATCH=1 && ab rcan k2b SR_SIDE_BATCH=2 && ab rcan k4b SR_SIDE_BATCH=4 && ab rcan k20b SR_SIDE_BATCH=20 && \
  ab swinir k1 SR_SIDE_BATCH=1 && ab swinir k2 SR_SIDE_BATCH=2 && ab swinir k6 SR_SIDE_BATCH=6 && \
  ab swinir k1b SR_SIDE_BATCH=1 && ab swinir k2b SR_SIDE_BATCH=2 && ab swinir k6b SR_SIDE_BATCH=6
