# round 3: the four bench lines (with this round's profiles/pmc_traffic.json) + 1x1 (linear) kernel micro
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_bench
timeout -k 10 120 python3 -u tools/bench_conv.py 32 0 "184,576,64,0,1;184,360,64,0,1;184,184,64,0,1" > gpurun_out/r3_bench/lin_micro.log 2>&1 || exit 3
for w in ${WORKLOADS:-edsr rcan swinir rrdb}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 > gpurun_out/r3_bench/bench_$w.json.log 2>&1 || exit 2
  echo "bench $w: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_bench/bench_$w.json.log | head -1)"
done
echo done
