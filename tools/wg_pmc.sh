#!/bin/bash
# SQ counters of the row-streaming wgrad kernel and the band fwd kernel (one pass)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/wg_pmc; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-include-regex "wgrad_ring|fwd_band" --output-format csv -d $OUT/p1 -o pmc -- python3 tools/bench_conv.py 32 0 "64,64,64,0" > $OUT/p1.log 2>&1
find $OUT -name "*.csv"
