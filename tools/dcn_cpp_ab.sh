#!/bin/bash
# A/B of the DCN scatter's channels per pass (SR_DCN_CPP 8 / 16 / 32): DCN parity tests under each,
# then the C5 op bench (fwd + bwd) under each, in one call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cpp
for c in 8 16 32; do
  SR_DCN_CPP=$c timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_dcn_ext_gpu.py > gpurun_out/cpp/t$c.log 2>&1 || { echo "tests cpp $c failed"; tail -5 gpurun_out/cpp/t$c.log; exit 2; }
  echo "cpp $c tests: $(tail -1 gpurun_out/cpp/t$c.log)"
done
for c in 8 16 32 8 16 32; do
  SR_DCN_CPP=$c timeout -k 10 200 python -u tools/bench_dcn.py --no-cpu > gpurun_out/cpp/b$c.log 2>&1 || exit 3
  echo "cpp $c: $(grep '^bf16' gpurun_out/cpp/b$c.log | cut -c1-60)"
done
