#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run: bash tools/prof_bench.sh <tag> <workload> [bench args]
# -> gpurun_out/<tag>/<workload>_kernel_stats.csv + bench log
set -o pipefail
TAG=$1; WL=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$WL -o run -- \
  python3 -u bench.py --workload $WL --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline "$@" > $OUT/bench_$WL.log 2>&1
rc=$?
f=$(find $OUT/prof_$WL -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/${WL}_kernel_stats.csv && rm -rf $OUT/prof_$WL
grep '^{"metric' $OUT/bench_$WL.log | cut -c1-200
exit $rc
