#!/bin/bash
# round 3 (third session): the four bench lines with this round's profiles/pmc_traffic.json, then the
# full GPU suite + smoke (what the driver runs at round end)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3c_bench gpurun_out/r3_full
for w in ${WORKLOADS:-edsr rcan swinir rrdb}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 > gpurun_out/r3c_bench/bench_$w.json.log 2>&1 || exit 2
  echo "bench $w: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3c_bench/bench_$w.json.log | head -1)"
done
[ "${SUITE:-1}" = 1 ] || exit 0
bash tools/gpu_r3_full.sh
