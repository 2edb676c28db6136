#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in rcan rrdb edsr; do echo "== $wl"; timeout -k 10 200 python -u tools/replay_gap.py --workload $wl --steps 8 || exit 1; done
