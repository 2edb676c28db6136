#!/bin/bash
# Round-6 pph column strips: tests, then the LR 256 sweep A/B (variant 77 = pp) and the headline step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s
mkdir -p $OUT
TEST_TIMEOUT=500 bash tools/gpu_tests.sh r6s_t tests/test_conv_gpu.py tests/test_workload_tiles_gpu.py -k "pph or strips or two_interval or edsr" || exit 1
for v in 0 77; do
  SR_CONV_VARIANT=$v timeout -k 10 300 python -u bench.py --workload edsr --lr-px 256 --batch 2 --steps 10 --warmup 3 \
    --no-cpu-baseline --no-parity > $OUT/lr256_v$v.json 2> $OUT/lr256_v$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/lr256_v$v.json').read().strip().splitlines()[-1]); print('lr256 v$v', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
timeout -k 10 300 python -u bench.py --workload edsr --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-trace \
  > $OUT/edsr64.json 2> $OUT/edsr64.err || exit 1
python3 -c "import json; d=json.loads(open('$OUT/edsr64.json').read().strip().splitlines()[-1]); print('edsr 64', d['ms_per_step'])"
