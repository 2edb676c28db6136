#!/bin/bash
# Round 4 session D: the DCN backward forms (tools/r4_dcn.sh), then SQ counters of the fused SwinIR
# attention half on the SwinIR-M bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/r4_dcn.sh || exit 1
echo "== swin_attn_block_fwd_kernel"
bash tools/pmc_kernel.sh swin_attn swin_attn_block_fwd_kernel python3 bench.py --workload swinir --steps 2 --warmup 1 \
  --no-cpu-baseline --no-parity || exit 1
