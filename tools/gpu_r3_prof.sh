# round 3: bench lines (all four workloads) + rocprofv3 evidence (kernel trace of the timed replays,
# FETCH / WRITE passes of each dominant kernel, plus RCAN's ring wgrad + slab reduce)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_prof
for w in edsr rcan swinir rrdb; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 > gpurun_out/r3_prof/bench_$w.json.log 2>&1 || exit 2
  echo "bench $w: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_prof/bench_$w.json.log | head -1)"
done
bash tools/profile_round.sh r03 "edsr:conv3x3_fwd_pph" "rcan:conv3x3_fwd_band" "swinir:conv3x3_wgrad_pp|wgrad_reduce_g" "rrdb:conv3x3_fwd_band" || exit 3
OUT=gpurun_out/prof_r03_rcan_ring; mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "conv3x3_wgrad_ring|wgrad_reduce_tr" --output-format csv -d $OUT/fetch -o pmc -- \
    python3 bench.py --workload rcan --steps 1 --warmup 1 --graph 0 --no-cpu-baseline --no-trace --no-parity > $OUT/bench_fetch.log 2>&1 || exit 4
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "conv3x3_wgrad_ring|wgrad_reduce_tr" --output-format csv -d $OUT/write -o pmc -- \
    python3 bench.py --workload rcan --steps 1 --warmup 1 --graph 0 --no-cpu-baseline --no-trace --no-parity > $OUT/bench_write.log 2>&1 || exit 5
cp -r gpurun_out/prof_r03_rcan/kt $OUT/kt
echo done
