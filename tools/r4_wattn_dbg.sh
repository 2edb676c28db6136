#!/bin/bash
# Window-attention backward forms: parity (bitwise / fp32-rounding vs the one-wave kernel, both
# reduce paths), then the micro-bench of every form (windows per wave x bias-gradient mode).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4wattn
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_swin_ops_gpu.py \
  -k "window_attention" > $OUT/tests2.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" $OUT/tests2.log | cut -c1-300 | tail -8; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u tools/bench_wattn.py --forms v1,u4a,u4,u2a,u2,u1a,u1 | tee $OUT/micro2.log
