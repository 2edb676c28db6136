cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6l
SR_HIP_LIB=abl/libA.so timeout -k 10 120 python -u tools/wgrad_dump.py gpurun_out/r6l/a.pt > gpurun_out/r6l/dump.log 2>&1 || exit 1
SR_HIP_LIB=abl/libB.so timeout -k 10 120 python -u tools/wgrad_dump.py gpurun_out/r6l/b.pt >> gpurun_out/r6l/dump.log 2>&1 || exit 1
python tools/wgrad_dump.py --cmp gpurun_out/r6l/a.pt gpurun_out/r6l/b.pt || exit 1
for L in A B A B; do
  SR_HIP_LIB=abl/lib$L.so timeout -k 10 120 python -u tools/bench_conv.py 32 0 "256,256,64,0" 2>/dev/null | grep wgrad | sed "s/^/$L /" || exit 1
done
SR_HIP_LIB=abl/libB.so TEST_TIMEOUT=600 bash tools/gpu_tests.sh r6l tests/test_conv_gpu.py tests/test_edsr_l_gpu.py tests/test_workload_tiles_gpu.py -k "wgrad or edsr" || exit 1
ABDIR=abl WORKLOADS=edsr ROUNDS=2 STEPS=20 bash tools/ab.sh
