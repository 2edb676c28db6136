#!/bin/bash
# phase cycles of the ring wgrad (stamps build tools/ab/libstamps.so): RCAN shape, EDSR-L shape at 256 / 512 blocks
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SR_HIP_LIB=tools/ab/libstamps.so
timeout -k 10 120 python3 tools/wg_stamps.py 32 64,64,64 || exit 1
for t in 256 512; do SR_RING_WIDE=$t timeout -k 10 120 python3 tools/wg_stamps.py 32 256,256,64 || exit 1; done
SR_RING_D=4 SR_RING_WIDE=256 timeout -k 10 120 python3 tools/wg_stamps.py 32 256,256,64 || exit 1
