#!/bin/bash
# Round 4 session C: fused SwinIR halves (parity + A/B), ring co-split parity + RCAN A/B, DCN SQ counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/r4_swin.sh || exit 1
OUT=gpurun_out/r4swin
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_conv_gpu.py -k "wgrad_halo" \
  > $OUT/halo.log 2>&1; rc=$?; tail -3 $OUT/halo.log; [ $rc -eq 0 ] || exit 1
for tag in cosplit base cosplit2 base2; do
  env $([ "${tag#cosplit}" != "$tag" ] && echo SR_RING_COSPLIT=1 || echo X=1) timeout -k 10 300 python -u bench.py --workload rcan \
    --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/rcan_$tag.log 2>&1 || { tail -20 $OUT/rcan_$tag.log; exit 1; }
  grep '^{"metric' $OUT/rcan_$tag.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.readline()); k=d['roofline'].get('kernels',{})
print('rcan $tag', d['ms_per_step'], {n[:34]:(v['avg_us'],v['ms_per_step']) for n,v in k.items() if 'wgrad' in n})"
done
bash tools/r4_dcn_sq.sh
