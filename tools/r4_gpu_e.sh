#!/bin/bash
# Round 4 session E: DCN backward forms (tools/r4_dcn.sh), fused SwinIR halves with branch-free stores
# (tools/r4_swin.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/r4_dcn.sh && bash tools/r4_swin.sh
