#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VAR=SR_CA_DOT VALUES="1 0" WL=rcan ROUNDS=3 bash tools/ab_vals.sh || exit 3
VAR=SR_RING_LA VALUES="3 5" WL=rrdb ROUNDS=1 bash tools/ab_vals.sh || exit 4
VAR=SR_RING_LA VALUES="3 5" WL=rcan ROUNDS=1 bash tools/ab_vals.sh || exit 4
