#!/bin/bash
# Kernel-row wgrad: parity tests, wgrad microbench against the pp kernel (variant 78), EDSR step over
# bias-role group sizes (SR_WG_ROW3; 0 = the pp kernel) -> gpurun_out/${1:-row3}/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-row3}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_workload_tiles_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "wgrad or edsr" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python -u tools/bench_conv.py 32 0,78,0,78 "256,256,64,0" > $OUT/micro.log 2>&1 || exit 1
grep wgrad $OUT/micro.log | python3 -c "import sys, json; print('wgrad us (variant 0 / 78)', [(json.loads(l)['v'], round(json.loads(l)['ms']*1e3, 1)) for l in sys.stdin])"
VAR=SR_WG_ROW3 VALS="${VALS:-unset 1 3 0}" WORKLOADS=edsr ROUNDS=${ROUNDS:-2} bash tools/ab_vals.sh ${1:-row3}
