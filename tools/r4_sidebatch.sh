#!/bin/bash
# Batched side-stream forks (ops.conv.side_batch): the async / DDP / RCAN / SwinIR GPU tests, then
# RCAN (graph + side stream) and SwinIR (eager + side stream) with one fork per block vs one per
# launch (SR_SIDE_BATCH=0; SwinIR's per-block batching is SR_STB_SIDE_BATCH=1), alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4sb
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_train_step_gpu.py \
  tests/test_ddp_gpu.py tests/test_workload_tiles_gpu.py > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" $OUT/tests.log | cut -c1-300 | tail -8; [ $rc -eq 0 ] || exit 1
ab() {  # $1 workload, $2 tag, rest: env
  wl=$1; tag=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/${wl}_$tag.log 2>&1 || { tail -20 $OUT/${wl}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${wl}_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$wl $tag', d['ms_per_step'])"
}
ab rcan batch X=1 && ab rcan perlaunch SR_SIDE_BATCH=0 && ab rcan batch2 X=1 && ab rcan perlaunch2 SR_SIDE_BATCH=0 && \
  ab rcan batch3 X=1 && ab rcan perlaunch3 SR_SIDE_BATCH=0 && \
  ab swinir stb SR_STB_SIDE_BATCH=1 && ab swinir base X=1 && ab swinir stb2 SR_STB_SIDE_BATCH=1 && ab swinir base2 X=1
