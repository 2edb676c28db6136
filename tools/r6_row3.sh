#!/bin/bash
# Kernel-row wgrad forms (SR_WG_ROW3_V): parity per form, wgrad microbench per form, EDSR step per form
# -> gpurun_out/${1:-row3}/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-row3}; mkdir -p $OUT
for v in ${FORMS:-0 1 2 3 4 5}; do
  SR_WG_ROW3_V=$v timeout -k 10 200 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "row3" > $OUT/tests_$v.log 2>&1 || { tail -30 $OUT/tests_$v.log; exit 1; }
  echo "form $v: $(tail -1 $OUT/tests_$v.log)"
done
for v in ${FORMS:-0 1 2 3 4 5}; do
  SR_WG_ROW3_V=$v timeout -k 10 120 python -u tools/bench_conv.py 32 0,0 "256,256,64,0" > $OUT/micro_$v.log 2>&1 || exit 1
  grep wgrad $OUT/micro_$v.log | python3 -c "import sys, json; print('form $v', [round(json.loads(l)['ms']*1e3, 1) for l in sys.stdin])"
done
VAR=SR_WG_ROW3_V VALS="${FORMS:-0 1 2 3 4 5}" WORKLOADS=edsr ROUNDS=${ROUNDS:-1} bash tools/ab_vals.sh ${1:-row3}
