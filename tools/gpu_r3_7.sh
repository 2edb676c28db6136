# round 3, GPU call 7: two-interval pph / wgrad schedules (variants 56 / 57 / 58): bitwise tests, A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_7
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "two_interval or pph" > gpurun_out/r3_7/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r3_7/tests.log)"
[ $rc -le 1 ] || exit 2
VAR=SR_CONV_VARIANT VALUES="0 56 57 58" WORKLOADS="edsr" ROUNDS=2 STEPS=20 timeout -k 10 900 bash tools/ab_val.sh || exit 3
VAR=SR_CONV_VARIANT VALUES="0 57" WORKLOADS="swinir" ROUNDS=1 STEPS=15 timeout -k 10 300 bash tools/ab_val.sh || exit 4
echo done
