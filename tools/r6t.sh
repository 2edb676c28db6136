#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6t; mkdir -p $OUT
TEST_TIMEOUT=400 bash tools/gpu_tests.sh r6t_t tests/test_conv_gpu.py tests/test_workload_tiles_gpu.py -k "strips or edsr" || exit 1
timeout -k 10 300 python -u bench.py --workload edsr --steps 10 --warmup 3 --no-cpu-baseline --no-parity > $OUT/edsr_traced.json 2> $OUT/edsr_traced.err || exit 1
python3 -c "import json; d=json.loads(open('$OUT/edsr_traced.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], json.dumps(d['roofline']['kernels'].get('conv3x3_fwd_band_kernel')))"
KNOB=SR_CONV_VARIANT VALS="0 76" WORKLOAD=edsr ROUNDS=2 bash tools/ab_knob.sh r6t_ab
