#!/bin/bash
# fused DCN forward: parity tests, then the C5 op bench with the fused kernel and without it (A/B
# in one call), then a kernel trace of the fused bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dcnf
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_dcn_ext_gpu.py > gpurun_out/dcnf/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/dcnf/pytest.log)"; [ $rc = 0 ] || exit 2
timeout -k 10 300 python -u tools/bench_dcn.py --out gpurun_out/dcnf/dcn_fused.json > gpurun_out/dcnf/bench_fused.log 2>&1 || exit 3
SR_DCN_FUSED=0 SR_DCN_COORD_WIN=0 timeout -k 10 300 python -u tools/bench_dcn.py --no-cpu --out gpurun_out/dcnf/dcn_unfused.json > gpurun_out/dcnf/bench_unfused.log 2>&1 || exit 4
grep -E "^(fp32|bf16)" gpurun_out/dcnf/bench_fused.log gpurun_out/dcnf/bench_unfused.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dcnf/kt -o kt -- python3 tools/bench_dcn.py --no-cpu > gpurun_out/dcnf/bench_kt.log 2>&1 || exit 5
RS=none timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "dcn_fwd_win" --output-format csv -d gpurun_out/dcnf/fetch -o pmc -- python3 tools/dcn_ablate.py > gpurun_out/dcnf/fetch.log 2>&1 || exit 6
RS=none timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "dcn_fwd_win" --output-format csv -d gpurun_out/dcnf/write -o pmc -- python3 tools/dcn_ablate.py > gpurun_out/dcnf/write.log 2>&1 || exit 7
echo done
