# round 3, GPU call 4: narrow-wgrad split sweep on RCAN and RRDB; conv tests of the ring kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_4
VAR=SR_RING_SPLITS VALUES="512 256 128 64" WORKLOADS="rcan rrdb" ROUNDS=2 STEPS=15 timeout -k 10 900 bash tools/ab_val.sh || exit 2
echo done
