#!/bin/bash
# Vector NCHW -> NHWC tile (nchw_to_nhwc_vec_kernel): bitwise tests, the DCN tests, then the C5 DCN
# op bench (its x / dy conversions) three times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4tr
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ops_gpu.py \
  tests/test_dcn_ext_gpu.py > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log | cut -c1-300; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/bench_dcn.py --no-cpu --modes bf16 --out $OUT/dcn_bench_$i.json > $OUT/bench_$i.log 2>&1 || { tail -5 $OUT/bench_$i.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/dcn_bench_$i.json'))['bf16']; print('dcn', d['fwd_ms'], d['fwd_bwd_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_dcn.py \
  --no-cpu --modes bf16 --iters 10 > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/dcn_kernel_stats.csv
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/dcn_kernel_stats.csv')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:8]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1))"
