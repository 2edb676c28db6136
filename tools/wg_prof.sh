#!/bin/bash
# per-kernel durations of the narrow wgrad (main kernel vs slab reduce), both forms
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/wg_prof; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/a -o kt -- python3 tools/bench_conv.py 32 0,37 "64,64,64,0" > $OUT/a.log 2>&1
find $OUT -name "*stats.csv"
