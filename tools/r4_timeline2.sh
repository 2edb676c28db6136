#!/bin/bash
# Kernel timelines of the RCAN and RRDB steps after the batched side-stream forks.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in rcan rrdb; do
  bash tools/r4_timeline.sh $wl _b > /dev/null 2>&1 || { echo "$wl failed"; tail -5 gpurun_out/r4tl_${wl}_b/bench.log; exit 1; }
  echo "== $wl"; grep -v "^    gap" gpurun_out/r4tl_${wl}_b/timeline.txt | tail -4
  grep "^    gap" gpurun_out/r4tl_${wl}_b/timeline.txt | tail -6
done
