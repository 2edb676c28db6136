#!/bin/bash
# LayerNorm backward fused into the dgrad GEMM (sr_linear_ln_bwd): parity against the two-launch path,
# the SwinIR model-level GPU tests, then the SwinIR-M bench SR_LN_BWD_FUSED=1 vs default, twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4lnb
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_swin_ops_gpu.py \
  -k "linear_ln_bwd" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" $OUT/tests.log | cut -c1-300 | tail -12; [ $rc -eq 0 ] || exit 1
for tag in fused unf fused2; do
  E=$([ "${tag#unf}" != "$tag" ] && echo 0 || echo 1)
  SR_LN_BWD_FUSED=$E timeout -k 10 300 python -u bench.py --workload swinir --steps 20 --warmup 5 --no-cpu-baseline \
    --no-parity > $OUT/swinir_$tag.log 2>&1 || { tail -20 $OUT/swinir_$tag.log; exit 1; }
  grep '^{"metric' $OUT/swinir_$tag.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.readline()); r=d['roofline'] or {}; k=r.get('kernels',{})
top=sorted(k.items(), key=lambda kv:-kv[1]['ms_per_step'])[:8]
print('swinir $tag', d['ms_per_step'], [(n[:34], v['avg_us'], v['ms_per_step']) for n,v in top])"
done
