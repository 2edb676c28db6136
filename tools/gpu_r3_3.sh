# round 3, GPU call 3: fused CA test, A/B of the fused channel-attention kernels on RCAN, RCAN rocprof
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_3
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_ca_fused_gpu.py "tests/test_workload_tiles_gpu.py::test_rcan_workload_tile_bf16" "tests/test_archs_gpu.py::test_arch_matches_golden_and_oracle_grads" > gpurun_out/r3_3/tests.log 2>&1
echo "tests rc=$?"
ENVVAR=SR_CA_UNFUSED WORKLOADS="rcan" ROUNDS=2 STEPS=20 timeout -k 10 600 bash tools/ab_env.sh || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_3/rcan_kt -o kt -- \
    python3 bench.py --workload rcan --steps 20 --warmup 3 --no-cpu-baseline --no-trace --no-parity > gpurun_out/r3_3/rcan_kt.log 2>&1 || exit 3
echo done
