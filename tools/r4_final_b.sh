#!/bin/bash
# Round 4 final B: rocprofv3 kernel-trace summaries + FETCH / WRITE PMC of each workload's dominant kernel
# (tools/profile_round.sh), plus the RCAN ring weight gradient and the SwinIR linear weight gradient
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh r04 edsr:conv3x3_fwd_pph rcan:conv3x3_fwd_band swinir:linear_wk_kernel rrdb:conv3x3_fwd_band || exit 1
for spec in rcan:"conv3x3_wgrad_ring|wgrad_reduce_tr" swinir:"linear_wgrad|wgrad_reduce"; do
  W=${spec%%:*}; KRE=${spec#*:}; OUT=gpurun_out/prof_r04_${W}_wg
  mkdir -p $OUT
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/fetch -o pmc -- \
    python3 bench.py --workload $W --steps 1 --warmup 1 --graph 0 --no-cpu-baseline --no-trace --no-parity > $OUT/f.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/write -o pmc -- \
    python3 bench.py --workload $W --steps 1 --warmup 1 --graph 0 --no-cpu-baseline --no-trace --no-parity > $OUT/w.log 2>&1 || exit 1
done
echo done
