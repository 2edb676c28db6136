#!/bin/bash
# Host time per train step and the GPU gap between steps (tools/replay_gap.py), unprofiled, for
# the given workloads (default: rcan rrdb edsr swinir).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in ${@:-rcan rrdb edsr swinir}; do
  echo "== $wl"; timeout -k 10 200 python -u tools/replay_gap.py --workload $wl --steps 8 || exit 1
done
