#!/bin/bash
# Window-attention backward at two waves per SIMD (wattn_bwd_mfma2_kernel): bitwise against the
# one-wave kernel and the fp64 attention tests, the SwinIR-M net tests, then the SwinIR-M bench with
# the new kernel (4 windows per wave, per-lane bias-gradient slot rows) vs SR_WATTN_BWD=1, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4wattn
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_swin_ops_gpu.py \
  tests/test_archs_gpu.py tests/test_train_step_gpu.py -k "window_attention or swinir or SwinIR" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" $OUT/tests.log | cut -c1-300 | tail -12; [ $rc -eq 0 ] || exit 1
for tag in u4 v1 u4b v1b u4c v1c; do
  V=$([ "${tag#v1}" != "$tag" ] && echo 1 || echo 2)
  SR_WATTN_BWD=$V timeout -k 10 300 python -u bench.py --workload swinir --steps 30 --warmup 5 --no-cpu-baseline \
    --no-parity > $OUT/swinir_$tag.log 2>&1 || { tail -20 $OUT/swinir_$tag.log; exit 1; }
  grep '^{"metric' $OUT/swinir_$tag.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.readline()); r=d['roofline'] or {}; k=r.get('kernels',{})
top=sorted(k.items(), key=lambda kv:-kv[1]['ms_per_step'])[:6]
print('swinir $tag', d['ms_per_step'], [(n[:30], v['avg_us'], v['ms_per_step']) for n,v in top])"
done
