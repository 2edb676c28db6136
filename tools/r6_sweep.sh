#!/bin/bash
# SURVEY §8 secondary sweep (LR 256 -> HR 1024) on the final build: EDSR (kernel-row wgrad on / off) and SwinIR
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sweep}; mkdir -p $OUT
for run in edsr_row3 edsr_pp swinir; do
  wl=${run%%_*}
  if [ $run = edsr_pp ]; then export SR_WG_ROW3=0; else unset SR_WG_ROW3; fi
  timeout -k 10 400 python -u bench.py --workload $wl --lr-px 256 --batch 2 > $OUT/$run.log 2> $OUT/$run.err || { tail -20 $OUT/$run.err; exit 1; }
  grep '^{"metric' $OUT/$run.log > $OUT/$run.json
  python3 -c "import json; d=json.load(open('$OUT/$run.json')); r=d['roofline']; print('$run', d['ms_per_step'], d['value'], d['config']['per_gpu_batch'], r['kernel'], r['frac'])"
done
