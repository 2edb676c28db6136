cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r6i
for L in E0 E1 E2 E3 E4 E0 E3 E4; do
  SR_HIP_LIB=abl/lib$L.so timeout -k 10 120 python -u tools/bench_conv.py 32 0 "256,256,64,0" 2>/dev/null | grep wgrad | sed "s/^/$L /" || exit 1
done > gpurun_out/r6i/micro.log
for r in 1 2; do for L in E0 E3 E4; do
  SR_HIP_LIB=abl/lib$L.so timeout -k 10 300 python -u bench.py --workload edsr --no-cpu-baseline --no-parity --no-trace --steps 20 --warmup 5 > gpurun_out/r6i/edsr_$L.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r6i/edsr_$L.json').read().strip().splitlines()[-1]); print('edsr $L', d['ms_per_step'])"
done; done > gpurun_out/r6i/step.log
timeout -k 10 600 python -u bench.py --lr-px 256 --batch 2 --steps 10 --warmup 3 --sub-workloads swinir --sub-cpu-seconds 8 --cpu-seconds 8 > gpurun_out/r6i/sweep.json 2> gpurun_out/r6i/sweep.err
