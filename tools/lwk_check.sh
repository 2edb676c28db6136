#!/bin/bash
# linear_wk_kernel: parity tests, wide-K 1x1 microbench on / off (SwinIR-M shapes, B 32), SwinIR step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lwk
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_swin_ops_gpu.py \
  tests/test_conv_gpu.py -k "wide_k or big_tile or linear" > gpurun_out/lwk/pytest.log 2>&1 || { tail -40 gpurun_out/lwk/pytest.log; exit 1; }
tail -1 gpurun_out/lwk/pytest.log
SH="184,576,64,0,1;184,360,64,0,1"
for v in 1 0; do
  SR_LWK=$v timeout -k 10 120 python3 -u tools/bench_conv.py 32 0 "$SH" > gpurun_out/lwk/micro_$v.log 2>&1 || { tail -5 gpurun_out/lwk/micro_$v.log; exit 2; }
  echo "SR_LWK=$v $(python3 -c "import sys,json; print([(d['k'], d['cin'], d['cout'], round(d['ms']*1000,1)) for d in map(json.loads, [l for l in open('gpurun_out/lwk/micro_$v.log') if l.startswith('{')])])")"
done
for r in 1 2; do
  for v in 1 0; do
    SR_LWK=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-trace --workload swinir --steps 10 --warmup 3 \
      > gpurun_out/lwk/b_${v}_$r.log 2>&1 || { tail -20 gpurun_out/lwk/b_${v}_$r.log; exit 3; }
    python3 -c "import json; d=json.loads(open('gpurun_out/lwk/b_${v}_$r.log').read().strip().splitlines()[-1]); print('swinir SR_LWK=$v', d['ms_per_step'], d.get('last_loss'))"
  done
done
