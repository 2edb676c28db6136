#!/bin/bash
# rocprofv3 passes for the round-1 bench (run from the repo root on the GPU box).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_under_kt.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv3x3_fwd_kernel --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace > $OUT/bench_pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv3x3_fwd_kernel --output-format csv -d $OUT/pmc_write -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace > $OUT/bench_pmc_write.log 2>&1
find $OUT -name "*.csv" | head -20
