#!/bin/bash
# Row-streaming wide wgrad (SR_RING_WIDE=<blocks>) A/B on the EDSR step inside one GPU call, after its
# parity test.  usage (GPU box): VALUES="0 256 512" ROUNDS=2 bash tools/ab_ring_wide.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rw
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
  -k "ring_wide or wgrad_halo" > gpurun_out/rw/pytest.log 2>&1 || { tail -30 gpurun_out/rw/pytest.log; exit 1; }
tail -1 gpurun_out/rw/pytest.log
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VALUES:-0 256}; do
    SR_RING_WIDE=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline ${TRACE:---no-trace} --workload ${WL:-edsr} \
      --steps ${STEPS:-10} --warmup 3 > gpurun_out/rw/b_${v}_$r.log 2>&1 || { tail -20 gpurun_out/rw/b_${v}_$r.log; exit 2; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rw/b_${v}_$r.log').read().strip().splitlines()[-1]); print('SR_RING_WIDE=$v', d['ms_per_step'], d.get('last_loss'))"
  done
done
