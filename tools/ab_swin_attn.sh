#!/bin/bash
# Fused-attention schedule flags (SR_SWIN_ATTN_V) at the C4 shape, one process per value, alternating
# rounds; then the SwinIR step for the given values.  usage (GPU box): VALS="0 1 3" bash tools/ab_swin_attn.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-swv}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2; do
  for v in ${VALS:-0 1 2 3 5 7}; do
    SR_SWIN_ATTN_V=$v timeout -k 10 120 python -u tools/bench_swin_fused.py 0 > $OUT/micro_v${v}_r$r.log 2>&1 || exit 1
    echo "v$v r$r $(tail -1 $OUT/micro_v${v}_r$r.log)"
  done
done
for r in 1 2; do
  for v in ${STEP_VALS:-0 1}; do
    SR_SWIN_ATTN_V=$v timeout -k 10 300 python -u bench.py --workload swinir --no-cpu-baseline --no-parity --steps 20 \
      --warmup 5 > $OUT/step_v${v}_r$r.json 2> $OUT/step_v${v}_r$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/step_v${v}_r$r.json').read().strip().splitlines()[-1]); print('step v$v r$r', d['ms_per_step'], d['swin_fused_attention']['attention_train'], d['swin_fused_attention']['attention_inference'])"
  done
done
