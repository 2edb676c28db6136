#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lwk3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_swin_ops_gpu.py \
  tests/test_conv_gpu.py -k "wide_k or big_tile or linear or ln" > gpurun_out/lwk3/pytest.log 2>&1 || { tail -40 gpurun_out/lwk3/pytest.log; exit 1; }
tail -1 gpurun_out/lwk3/pytest.log
VAR=SR_LN_UNFUSED VALUES="0 1" WL=swinir ROUNDS=2 bash tools/ab_vals.sh || exit 3
