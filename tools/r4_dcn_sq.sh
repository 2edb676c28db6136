#!/bin/bash
# SQ counters of the fused DCN backward kernels on the C5 op bench (tools/pmc_kernel.sh: one rocprofv3
# pass per counter group, one kernel at a time)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in dcn_coord_dy dcn_gradx_dy; do
  echo "== $k"
  bash tools/pmc_kernel.sh $k "$k" python3 tools/bench_dcn.py --no-cpu --modes bf16 --iters 2 || exit 1
done
