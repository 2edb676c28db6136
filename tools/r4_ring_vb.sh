#!/bin/bash
# Round 4: ring wgrad with two row groups per 8-wave block (Cout <= 32) -- parity, then RRDB / RCAN A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4_ring
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_conv_gpu.py -k "halo_vs_fp64 or ring" \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_workload_tiles_gpu.py -k rrdb_workload \
  > $OUT/tile.log 2>&1 || { tail -30 $OUT/tile.log; exit 1; }
tail -2 $OUT/tile.log
for wl in rrdb rcan; do
  for vb in 2 1 2 1; do
    SR_RING_VB=$vb timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-trace \
      > $OUT/${wl}_vb$vb.log 2>&1 || { tail -20 $OUT/${wl}_vb$vb.log; exit 1; }
    grep '^{"metric' $OUT/${wl}_vb$vb.log | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$wl vb$vb', d['ms_per_step'])"
  done
done
