#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hps
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
  tests/test_workload_tiles_gpu.py tests/test_archs_gpu.py -k "pixel_shuffled or halo or rcan or swinir or conv3x3_fwd_bwd" > gpurun_out/hps/pytest.log 2>&1 || { tail -30 gpurun_out/hps/pytest.log; exit 1; }
tail -1 gpurun_out/hps/pytest.log
for v in 1 0; do
  SR_HALO_PS=$v timeout -k 10 120 python3 -u tools/bench_conv.py 32 0 "64,256,64,2;64,256,128,2" > gpurun_out/hps/micro_$v.log 2>&1 || exit 2
  echo "SR_HALO_PS=$v $(python3 -c "import json; print([(d['k'], d['hw'], round(d['ms']*1000,1)) for d in map(json.loads, [l for l in open('gpurun_out/hps/micro_$v.log') if l.startswith('{')]) if d['k']=='dgrad'])")"
done
VAR=SR_HALO_PS VALUES="1 0" WL=rcan ROUNDS=2 bash tools/ab_vals.sh || exit 3
VAR=SR_HALO_PS VALUES="1 0" WL=swinir ROUNDS=2 bash tools/ab_vals.sh || exit 3
