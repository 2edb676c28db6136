#!/bin/bash
# round 3: ring wgrad early issue / lookahead and the fused CA dot partials -- parity tests, ring stamps, RCAN / RRDB A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rab
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
  tests/test_workload_tiles_gpu.py tests/test_train_step_gpu.py -k "dot or ring or halo or rcan or async or wgrad" \
  > gpurun_out/rab/pytest.log 2>&1 || { tail -40 gpurun_out/rab/pytest.log; exit 1; }
tail -1 gpurun_out/rab/pytest.log
VAR=SR_RING_EARLY VALUES="1 0" WL=rcan ROUNDS=2 bash tools/ab_vals.sh || exit 2
VAR=SR_CA_DOT VALUES="1 0" WL=rcan ROUNDS=1 bash tools/ab_vals.sh || exit 3
VAR=SR_RING_LA VALUES="3 5" WL=rcan ROUNDS=1 bash tools/ab_vals.sh || exit 4
VAR=SR_RING_EARLY VALUES="1 0" WL=rrdb ROUNDS=1 bash tools/ab_vals.sh || exit 5
