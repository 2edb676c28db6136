#!/bin/bash
# Per-round rocprofv3 evidence for bench.py, one workload at a time (GPU box, repo root):
#   1. --kernel-trace --stats of the bench step as the bench line runs it (HIP graph on), 20 timed
#      steps after 3 warm-up steps, without the traced step / relaunch passes / parity net, so the
#      averages are those of the timed replays
#   2. FETCH_SIZE of the dominant kernel(s) (own pass, eager steps, --pmc only)
#   3. WRITE_SIZE of the same (own pass)
# then, back in the build container:
#   python3 tools/pmc_summary.py <tag> <workload> <kernel-regex> gpurun_out/prof_<tag>_<workload> <bench-kernel> [<time-regex>]
# folds them into profiles/<tag>/ (+ profiles/pmc_traffic.json).
# usage: bash tools/profile_round.sh <tag> <workload>:<pmc-kernel-regex> [...]
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "$@"; do
  W=${spec%%:*}; KRE=${spec#*:}
  OUT=gpurun_out/prof_${TAG}_$W
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
    python3 bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-trace --no-parity > $OUT/bench_under_kt.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/fetch -o pmc -- \
    python3 bench.py --workload $W --steps 1 --warmup 1 --graph 0 --no-cpu-baseline --no-trace --no-parity > $OUT/bench_fetch.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/write -o pmc -- \
    python3 bench.py --workload $W --steps 1 --warmup 1 --graph 0 --no-cpu-baseline --no-trace --no-parity > $OUT/bench_write.log 2>&1
done
