# round 3, GPU call 6: wide-K lin kernel (tests + SwinIR A/B vs variant 55), ring depth tests + sweep
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_6
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_swin_ops_gpu.py "tests/test_workload_tiles_gpu.py::test_swinir_m_workload_tile_bf16" "tests/test_archs_gpu.py::test_swinir_bf16_c4_shape" > gpurun_out/r3_6/tests_lin.log 2>&1
echo "lin tests rc=$? $(tail -1 gpurun_out/r3_6/tests_lin.log)"
VAR=SR_CONV_VARIANT VALUES="0 55" WORKLOADS="swinir" ROUNDS=2 STEPS=15 timeout -k 10 600 bash tools/ab_val.sh || exit 2
for d in 3 4; do
  SR_RING_D=$d timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "wgrad_halo or wgrad_bf16 or rgb_head" > gpurun_out/r3_6/tests_d$d.log 2>&1
  echo "ring tests D=$d rc=$? $(tail -1 gpurun_out/r3_6/tests_d$d.log)"
done
VAR=SR_RING_D VALUES="2 3 4" WORKLOADS="rcan rrdb" ROUNDS=2 STEPS=15 timeout -k 10 900 bash tools/ab_val.sh || exit 3
echo done
