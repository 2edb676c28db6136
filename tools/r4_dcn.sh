#!/bin/bash
# Round 4 DCN session: parity of the fused backward (sr_dcn_bwd_fused) and every DCN test, then the
# C5 op bench fused vs the dcols path (SR_DCN_BWD_FUSED=0), a rocprofv3 kernel-trace summary of the
# bf16 bench, and FETCH / WRITE PMC passes over the same command (one pass each).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4dcn
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_ops_gpu.py \
  tests/test_dcn_ext_gpu.py -k "dcn or DCN or deform" > $OUT/tests.log 2>&1; rc=$?
grep -E "rel err|passed|failed|Error" $OUT/tests.log | cut -c1-250 | tail -30; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_dcn.py --no-cpu --modes bf16 --out $OUT/dcn_bench.json > $OUT/bench_fused.log 2>&1 \
  && grep '^bf16' $OUT/bench_fused.log || exit 1
SR_DCN_BWD_FUSED=0 timeout -k 10 300 python -u tools/bench_dcn.py --no-cpu --modes bf16 > $OUT/bench_dcols.log 2>&1 \
  && grep '^bf16' $OUT/bench_dcols.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 tools/bench_dcn.py --no-cpu --modes bf16 \
  --iters 10 > $OUT/prof.log 2>&1 || exit 1
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/dcn_kernel_stats.csv
python3 -c "
import csv
r=list(csv.DictReader(open('$OUT/dcn_kernel_stats.csv')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:12]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1))"
for pmc in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc_$pmc -o run -- python3 tools/bench_dcn.py --no-cpu --modes bf16 \
    --iters 4 > $OUT/pmc_$pmc.log 2>&1 || exit 1
done
echo done
