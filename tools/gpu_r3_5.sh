# round 3, GPU call 5: ring wgrad pipeline depth (SR_RING_D): correctness at D=3/4, then a sweep
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_5
for d in 3 4; do
  SR_RING_D=$d timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "wgrad_halo or wgrad_bf16 or rgb_head" > gpurun_out/r3_5/tests_d$d.log 2>&1
  echo "tests D=$d rc=$? $(tail -1 gpurun_out/r3_5/tests_d$d.log)"
done
VAR=SR_RING_D VALUES="2 3 4" WORKLOADS="rcan rrdb" ROUNDS=2 STEPS=15 timeout -k 10 900 bash tools/ab_val.sh || exit 2
echo done
