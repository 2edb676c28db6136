#!/bin/bash
# GPU box: every BASELINE workload through bench.py (one JSON line each) -> gpurun_out/bench_<w>.log
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in ${WORKLOADS:-edsr rcan swinir rrdb}; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload $w --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench_$w.log 2>&1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$w.log').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('$w', d['value'], d['ms_per_step'], [(n, v['ms_per_step']) for n, v in list(k.items())[:6]])"
done
