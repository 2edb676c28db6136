#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/red
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
  -k "reduce_t9 or wgrad_bf16 or pp_bitwise or tr3" > gpurun_out/red/pytest.log 2>&1 || { tail -30 gpurun_out/red/pytest.log; exit 1; }
tail -1 gpurun_out/red/pytest.log
for v in 1 0; do
  SR_RED_T9=$v timeout -k 10 120 python3 -u tools/bench_conv.py 32 0 "256,256,64,0;256,1024,64,2" > gpurun_out/red/micro_$v.log 2>&1 || exit 2
  echo "SR_RED_T9=$v $(python3 -c "import json; print([(d['k'], d['cout'], round(d['ms']*1000,1)) for d in map(json.loads, [l for l in open('gpurun_out/red/micro_$v.log') if l.startswith('{')]) if d['k']=='wgrad'])")"
done
VAR=SR_RED_T9 VALUES="1 0" WL=edsr ROUNDS=3 bash tools/ab_vals.sh || exit 3
