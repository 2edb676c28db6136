#!/bin/bash
# Kernel timelines (tools/timeline.py) of the EDSR, RCAN and RRDB bench steps (their default step modes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in edsr rcan rrdb; do
  bash tools/r4_timeline.sh $wl > /dev/null 2>&1 || { echo "$wl failed"; tail -5 gpurun_out/r4tl_$wl/bench.log; exit 1; }
  echo "== $wl"; grep -v "^    gap" gpurun_out/r4tl_$wl/timeline.txt | tail -4
  grep "^    gap" gpurun_out/r4tl_$wl/timeline.txt | tail -6
done
