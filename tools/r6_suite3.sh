#!/bin/bash
# the default bench line (the driver's command) three times, and the kpad / swin tests first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-suite3}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_workload_tiles_gpu.py tests/test_swin_fused_gpu.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider -k "kpad or swinir or swin" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  timeout -k 10 780 python -u bench.py > $OUT/bench_$r.log 2> $OUT/bench_$r.err || { tail -20 $OUT/bench_$r.err; exit 1; }
  grep '^{"metric' $OUT/bench_$r.log > $OUT/bench_$r.json
  python3 -c "
import json; d=json.load(open('$OUT/bench_$r.json'))
print('run $r edsr', d['ms_per_step'], ' '.join(f'{k} {s[\"ms_per_step\"]}' for k, s in d['sub_records'].items()))"
done
