#!/bin/bash
# Round 4 closing call: the whole GPU suite, smoke and the four bench lines (tools/r4_final_a.sh),
# then the EDSR ring-wgrad split / depth A/B and the SwinIR host-vs-GPU step times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/r4_final_a.sh || exit 1
bash tools/r4_edsr_ring.sh
