#!/bin/bash
# round 3, last session: the DCN scatter A/B (channels per pass), then the four bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/dcn_cpp_ab.sh || exit 2
SUITE=0 bash tools/gpu_r3c_bench.sh || exit 3
