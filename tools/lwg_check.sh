#!/bin/bash
# linear_wgrad_kernel: parity tests, 1x1 microbench (SwinIR-M shapes, B 32) on / off, SwinIR step A/B.
# usage (GPU box): bash tools/lwg_check.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lwg
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
  -k "linear_wgrad or ring_wide or wgrad" > gpurun_out/lwg/pytest.log 2>&1 || { tail -40 gpurun_out/lwg/pytest.log; exit 1; }
tail -1 gpurun_out/lwg/pytest.log
SH="184,576,64,0,1;192,184,64,0,1;184,360,64,0,1;360,184,64,0,1"
for v in 1 0; do
  SR_LWG=$v timeout -k 10 120 python3 -u tools/bench_conv.py 32 0 "$SH" > gpurun_out/lwg/micro_$v.log 2>&1 || { tail -5 gpurun_out/lwg/micro_$v.log; exit 2; }
  echo "SR_LWG=$v $(grep wgrad1x1 gpurun_out/lwg/micro_$v.log | python3 -c "import sys,json; print([(json.loads(l)['cin'], json.loads(l)['cout'], round(json.loads(l)['ms']*1000,1)) for l in sys.stdin])")"
done
for t in ${TARGETS:-128 512}; do
  SR_LWG_T=$t timeout -k 10 120 python3 -u tools/bench_conv.py 32 0 "$SH" > gpurun_out/lwg/micro_t$t.log 2>&1 || exit 2
  echo "SR_LWG_T=$t $(grep wgrad1x1 gpurun_out/lwg/micro_t$t.log | python3 -c "import sys,json; print([(json.loads(l)['cin'], json.loads(l)['cout'], round(json.loads(l)['ms']*1000,1)) for l in sys.stdin])")"
done
for r in 1 2; do
  for v in 1 0; do
    SR_LWG=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-trace --workload swinir --steps 10 --warmup 3 \
      > gpurun_out/lwg/b_${v}_$r.log 2>&1 || { tail -20 gpurun_out/lwg/b_${v}_$r.log; exit 3; }
    python3 -c "import json; d=json.loads(open('gpurun_out/lwg/b_${v}_$r.log').read().strip().splitlines()[-1]); print('swinir SR_LWG=$v', d['ms_per_step'], d.get('last_loss'))"
  done
done
