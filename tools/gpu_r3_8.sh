# round 3, GPU call 8: deep B prefetch in the pph kernel (variant 60): bitwise tests, EDSR A/B; full suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_8
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "two_interval or pph" > gpurun_out/r3_8/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r3_8/tests.log)"
[ $rc -le 1 ] || exit 2
VAR=SR_CONV_VARIANT VALUES="0 60" WORKLOADS="edsr" ROUNDS=3 STEPS=20 timeout -k 10 900 bash tools/ab_val.sh || exit 3
bash tools/gpu_r3_full.sh
