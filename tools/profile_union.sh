#!/bin/bash
# Per-round rocprofv3 evidence, one workload at a time (GPU box, repo root), like tools/profile_round.sh
# but with ONE union kernel regex per workload for the FETCH_SIZE / WRITE_SIZE passes, so several
# kernels' traffic comes from the same two passes (split by tools/pmc_summary.py's kernel / time regexes):
#   bash tools/profile_union.sh <tag> <workload>:<union-regex> [...]
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "$@"; do
  W=${spec%%:*}; KRE=${spec#*:}
  OUT=gpurun_out/prof_${TAG}_$W
  mkdir -p $OUT
  echo "$W: kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
    python3 bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-trace --no-parity > $OUT/bench_under_kt.log 2>&1
  echo "$W: FETCH_SIZE"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/fetch -o pmc -- \
    python3 bench.py --workload $W --steps 1 --warmup 1 --graph 0 --no-cpu-baseline --no-trace --no-parity > $OUT/bench_fetch.log 2>&1
  echo "$W: WRITE_SIZE"
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/write -o pmc -- \
    python3 bench.py --workload $W --steps 1 --warmup 1 --graph 0 --no-cpu-baseline --no-trace --no-parity > $OUT/bench_write.log 2>&1
done
