#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lwk2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_swin_ops_gpu.py \
  tests/test_conv_gpu.py tests/test_workload_tiles_gpu.py -k "wide_k or big_tile or linear or swinir or dcn" > gpurun_out/lwk2/pytest.log 2>&1 || { tail -40 gpurun_out/lwk2/pytest.log; exit 1; }
tail -1 gpurun_out/lwk2/pytest.log
SH="184,184,64,0,1;184,360,64,0,1;192,184,64,0,1"
for v in 0 192; do
  SR_LWK_MINK=$v timeout -k 10 120 python3 -u tools/bench_conv.py 32 0 "$SH" > gpurun_out/lwk2/micro_$v.log 2>&1 || { tail -5 gpurun_out/lwk2/micro_$v.log; exit 2; }
  echo "MINK=$v $(python3 -c "import json; print([(d['k'], d['cin'], d['cout'], round(d['ms']*1000,1)) for d in map(json.loads, [l for l in open('gpurun_out/lwk2/micro_$v.log') if l.startswith('{')]) if d['k'] != 'wgrad1x1'])")"
done
VAR=SR_LWK_MINK VALUES="0 192" WL=swinir ROUNDS=2 bash tools/ab_vals.sh || exit 3
