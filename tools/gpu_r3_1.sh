set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_workload_tiles_gpu.py tests/test_srrs_model_gpu.py tests/test_ddp_gpu.py tests/test_train_entry_gpu.py -s > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 3 --workload rcan > gpurun_out/b_rcan_dp2_gloo.log 2>&1
echo "bench rc=$?"
