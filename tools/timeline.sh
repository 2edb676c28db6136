#!/bin/bash
# Kernel timeline of the SwinIR-M (or other) bench step: rocprofv3 kernel trace of a short bench run,
# then tools/timeline.py: per step, GPU busy time (union of kernel intervals), idle gaps, overlap.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
WL=${1:-swinir}
TAG=${2:-}
shift 2 2>/dev/null || shift $#
OUT=gpurun_out/tl_$WL$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --workload $WL \
  --steps 10 --warmup 3 --no-cpu-baseline --no-parity "$@" > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1); cp "$f" $OUT/kernel_trace.csv
python3 tools/timeline.py $OUT/kernel_trace.csv | tee $OUT/timeline.txt
