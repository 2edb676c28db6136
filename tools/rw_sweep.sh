#!/bin/bash
# Wide row-streaming wgrad sweep on the EDSR-L body shape (B 32, 256 -> 256, 64^2): block target x
# steps in flight, microbench (tools/bench_conv.py, HIP events).  usage (GPU box): bash tools/rw_sweep.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rw
SHAPES=${SHAPES:-"256,256,64,0"}
for t in ${TARGETS:-0 256 512 1024}; do
  for dd in ${DEPTHS:-2 3 4}; do
    [ "$t" = 0 ] && [ "$dd" != 2 ] && continue
    SR_RING_WIDE=$t SR_RING_D=$dd timeout -k 10 120 python3 -u tools/bench_conv.py 32 0 "$SHAPES" \
      > gpurun_out/rw/sw_${t}_${dd}.log 2>&1 || { tail -5 gpurun_out/rw/sw_${t}_${dd}.log; exit 1; }
    echo "T=$t D=$dd $(grep wgrad gpurun_out/rw/sw_${t}_${dd}.log | python3 -c "import sys,json; print([ (json.loads(l)['cout'], round(json.loads(l)['ms']*1000,1)) for l in sys.stdin])")"
  done
done
