#!/bin/bash
# rocprofv3 passes for bench.py (run from the repo root on the GPU box):
#   1. kernel trace + stats (per-kernel average durations)
#   2./3. FETCH_SIZE / WRITE_SIZE of the dominant kernel, each in its own pass
# usage: bash tools/profile.sh <tag> [kernel-regex]
set -e
TAG=${1:-r01}
KRE=${2:-conv3x3_fwd_pp_kernel}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_under_kt.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace > $OUT/bench_pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc_write -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace > $OUT/bench_pmc_write.log 2>&1
find $OUT -name "*.csv"
