#!/bin/bash
# round 3 (third session): rocprofv3 evidence for the four bench lines -- kernel trace of the timed
# steps + FETCH / WRITE passes of each workload's dominant kernel (SwinIR's picked from its bench line).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3c
timeout -k 10 400 python -u bench.py --workload swinir --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/r3c/swinir_pick.log 2>&1 || exit 2
K=$(python3 -c "import json; print(json.loads(open('gpurun_out/r3c/swinir_pick.log').read().strip().splitlines()[-1])['roofline']['kernel'])")
echo "swinir dominant: $K"
case "$K" in
  linear_wgrad_kernel+reduce) SRE="linear_wgrad_kernel|wgrad_reduce" ;;
  linear_wk_kernel) SRE="linear_wk_kernel" ;;
  conv3x3_lin_kernel+ln) SRE="conv3x3_lin_kernel<.*true>" ;;
  *) SRE="conv3x3_lin_kernel" ;;
esac
echo "$K" > gpurun_out/r3c/swinir_kernel.txt
echo "$SRE" > gpurun_out/r3c/swinir_regex.txt
bash tools/profile_round.sh r03c "edsr:conv3x3_fwd_pph" "rcan:conv3x3_fwd_band" "swinir:$SRE" "rrdb:conv3x3_fwd_band" || exit 3
echo done
