#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TEST_TIMEOUT=500 bash tools/gpu_tests.sh r6v_t tests/test_conv_gpu.py tests/test_workload_tiles_gpu.py tests/test_train_step_gpu.py -k "wgrad or edsr or swinir or bitwise or reduce" || exit 1
ABDIR=abl WORKLOADS="edsr" ROUNDS=3 STEPS=20 bash tools/ab.sh || exit 1
ABDIR=abl WORKLOADS="swinir" ROUNDS=1 STEPS=20 bash tools/ab.sh
