#!/bin/bash
# lin kernel: timing at the SwinIR qkv / fc1 / proj shapes, then SQ counters (one pass)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/lin_pmc; mkdir -p $OUT
timeout -k 10 120 python3 tools/bench_conv.py 32 0 "184,552,64,0,1;184,368,64,0,1;184,184,64,0,1" > $OUT/time.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES --kernel-include-regex "lin_kernel" --output-format csv -d $OUT/p1 -o pmc -- python3 tools/bench_conv.py 32 0 "184,552,64,0,1" > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "lin_kernel" --output-format csv -d $OUT/p2 -o pmc -- python3 tools/bench_conv.py 32 0 "184,552,64,0,1" > $OUT/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "lin_kernel" --output-format csv -d $OUT/p3 -o pmc -- python3 tools/bench_conv.py 32 0 "184,552,64,0,1" > $OUT/p3.log 2>&1
