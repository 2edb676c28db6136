#!/bin/bash
# GPU box, end of a round: full GPU suite, smoke, then every workload's bench line with its CPU
# baseline and parity (default bench.py flags) -> gpurun_out/final_<w>.json
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
for w in edsr rcan swinir rrdb; do
  timeout -k 10 400 python -u bench.py --workload $w --steps ${STEPS:-10} --warmup 3 > gpurun_out/final_$w.log 2>&1 || exit 1
  grep '^{' gpurun_out/final_$w.log | tail -1 > gpurun_out/final_$w.json
  python3 -c "import json; d=json.load(open('gpurun_out/final_$w.json')); print('$w', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None, d['parity']['psnr_bf16_db'])"
done
