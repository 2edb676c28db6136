#!/bin/bash
# Round-6 closing evidence, part 2: rocprofv3 kernel stats + one FETCH_SIZE and one WRITE_SIZE pass per
# workload over a union kernel regex (tools/profile_union.sh), folded on the CPU by tools/pmc_summary.py
set -e
bash tools/profile_union.sh ${1:-r6f} \
  "edsr:conv3x3_fwd_pph|conv3x3_wgrad_row3|conv3x3_wgrad_pp|wgrad_reduce_g" \
  "rcan:conv3x3_fwd_band|conv3x3_wgrad_ring|wgrad_reduce_tr" \
  "swinir:linear_wk_kernel|swin_attn_block|linear_wgrad|wgrad_reduce_g|wgrad_reduce4" \
  "rrdb:conv3x3_fwd_band|conv3x3_wgrad_ring|wgrad_reduce_tr"
