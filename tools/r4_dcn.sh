#!/bin/bash
# Round 4 DCN session: parity of the fused backward forms (sr_dcn_bwd_fused) and every DCN test, the
# C5 op bench for each backward form (eight-channel kernels with the int32 / int64 fixed-point scatter
# image, four-channel kernels, the dcols path), then a rocprofv3 kernel-trace summary of the default form and
# FETCH / WRITE PMC passes over the same command (one pass each).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4dcn
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_ops_gpu.py \
  tests/test_dcn_ext_gpu.py -k "dcn or DCN or deform" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error" $OUT/tests.log | cut -c1-250 | tail -8; [ $rc -eq 0 ] || exit 1
bd() {  # $1 tag, rest: env
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u tools/bench_dcn.py --no-cpu --modes bf16 --out $OUT/dcn_bench_$tag.json \
    > $OUT/bench_$tag.log 2>&1 || { tail -5 $OUT/bench_$tag.log; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/dcn_bench_$tag.json'))['bf16']; print('$tag', d['fwd_ms'], d['fwd_bwd_ms'])"
}
bd i32 X=1 && bd i64 SR_DCN_GX_FX=64 && bd dcols SR_DCN_BWD_FUSED=0 && bd i32_b X=1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_dcn.py \
  --no-cpu --modes bf16 --iters 10 > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/dcn_kernel_stats.csv
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/dcn_kernel_stats.csv')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:12]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1))"
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "dcn_" --output-format csv -d $OUT/pmc_$pmc -o run -- \
    python3 tools/bench_dcn.py --no-cpu --modes bf16 --iters 4 > $OUT/pmc_$pmc.log 2>&1 || exit 1
done
echo done
