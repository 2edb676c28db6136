#!/bin/bash
# RCAN channel-attention A/B: fused squeeze-MLP + apply kernels (default) vs the separate MLP launch
# (SR_CA_UNFUSED=1), with and without the dgrad-epilogue dot partials (SR_CA_DOT=1); then the DCN
# forms again (scatter operands one tap ahead)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4ca
mkdir -p $OUT
for tag in base unf dot unfdot base2 unfdot2; do
  case $tag in base*) E=X=1;; unfdot*) E="SR_CA_UNFUSED=1 SR_CA_DOT=1";; unf) E=SR_CA_UNFUSED=1;; dot) E=SR_CA_DOT=1;; esac
  env $E timeout -k 10 300 python -u bench.py --workload rcan --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/rcan_$tag.log 2>&1 || { tail -20 $OUT/rcan_$tag.log; exit 1; }
  grep '^{"metric' $OUT/rcan_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('rcan $tag', d['ms_per_step'])"
done
bash tools/r4_dcn.sh
