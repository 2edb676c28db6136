#!/bin/bash
# One-row halo tiles for the wide W-256 convs (SR_HALO_W256=1: the HR conv_last dgrads, RRDB's 256^2
# dgrad) instead of the 256x256 pp / generic tile kernels: parity, then EDSR / RCAN / RRDB A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4h256
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_conv_gpu.py \
  -k "halo" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log | cut -c1-200; [ $rc -eq 0 ] || exit 1
ab() {  # $1 workload, $2 tag, rest: env
  wl=$1; tag=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/${wl}_$tag.log 2>&1 || { tail -20 $OUT/${wl}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${wl}_$tag.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.readline()); k=d['roofline']['kernels']
print('$wl $tag', d['ms_per_step'], [(n, v['avg_us'], v['calls']) for n, v in k.items() if n.startswith('conv3x3_fwd_pp_') or 'halo' in n or n.startswith('conv3x3_fwd_kernel')])"
}
for wl in edsr rcan rrdb; do
  ab $wl base X=1 && ab $wl h256 SR_HALO_W256=1 && ab $wl base2 X=1 && ab $wl h256b SR_HALO_W256=1 || exit 1
done
