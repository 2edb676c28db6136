#!/bin/bash
# Band kernel at two blocks per CU (W 64 forms, band_occ): the conv / RCAN GPU tests, then RCAN and
# the RCAN-shape band micro timing with SR_BAND_2PC=1 (default) vs 0, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4band2
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_ca_fused_gpu.py tests/test_workload_tiles_gpu.py -k "band or rcan or RCAN or ca" > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log | cut -c1-300; [ $rc -eq 0 ] || exit 1
ab() {  # $1 workload, $2 tag, rest: env
  wl=$1; tag=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline --no-parity \
    > $OUT/${wl}_$tag.log 2>&1 || { tail -20 $OUT/${wl}_$tag.log; return 1; }
  grep '^{"metric' $OUT/${wl}_$tag.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.readline()); r=d['roofline'] or {}; k=r.get('kernels',{})
b=k.get('conv3x3_fwd_band_kernel',{})
print('$wl $tag', d['ms_per_step'], 'band avg us', b.get('avg_us'), 'ms/step', b.get('ms_per_step'))"
}
ab rcan two X=1 && ab rcan one SR_BAND_2PC=0 && ab rcan two2 X=1 && ab rcan one2 SR_BAND_2PC=0 && \
  ab rcan two3 X=1 && ab rcan one3 SR_BAND_2PC=0
