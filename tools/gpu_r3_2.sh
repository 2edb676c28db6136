# round 3, GPU call 2: DDP graph-segment tests, fused channel-attention kernels, RCAN at its tile,
# the N=2 gloo bench rehearsal, RCAN bench, DCNv2 at the C5 op config
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_2
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_ca_fused_gpu.py tests/test_ddp_gpu.py "tests/test_workload_tiles_gpu.py::test_rcan_workload_tile_bf16" "tests/test_train_step_gpu.py::test_async_wgrad_bitwise_equals_sync" tests/test_archs_gpu.py -s > gpurun_out/r3_2/tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python bench.py --workload rcan --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3_2/b_rcan.log 2>&1
echo "bench rcan rc=$?"
SR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 3 --workload rcan --no-trace > gpurun_out/r3_2/b_rcan_dp2_gloo.log 2>&1
echo "bench dp2 rc=$?"
timeout -k 10 300 python -u tools/bench_dcn.py --out gpurun_out/r3_2/dcn_bench.json > gpurun_out/r3_2/dcn.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_2/dcn_kt -o kt -- python3 tools/bench_dcn.py --no-cpu --iters 10 > gpurun_out/r3_2/dcn_kt.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "dcn_|conv3x3" --output-format csv -d gpurun_out/r3_2/dcn_fetch -o pmc -- python3 tools/bench_dcn.py --no-cpu --iters 2 > gpurun_out/r3_2/dcn_fetch.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "dcn_|conv3x3" --output-format csv -d gpurun_out/r3_2/dcn_write -o pmc -- python3 tools/bench_dcn.py --no-cpu --iters 2 > gpurun_out/r3_2/dcn_write.log 2>&1 || exit 6
echo done
