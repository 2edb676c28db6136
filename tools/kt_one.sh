#!/bin/bash
# bench line (with its per-kernel trace) + rocprofv3 --kernel-trace --stats of the timed steps, one workload.
# usage (GPU box): WL=swinir TAG=x bash tools/kt_one.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/kt_${TAG:-x}_${WL:-swinir}; mkdir -p $OUT
timeout -k 10 400 python -u bench.py --workload ${WL:-swinir} --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json.log 2>&1 || { tail -5 $OUT/bench.json.log; exit 2; }
echo "bench: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json.log | head -1)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
  python3 bench.py --workload ${WL:-swinir} --steps 20 --warmup 3 --no-cpu-baseline --no-trace --no-parity > $OUT/bench_under_kt.log 2>&1 || exit 3
echo done
