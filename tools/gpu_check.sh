#!/bin/bash
# GPU box: parity tests, smoke, bench (each step under its own time limit; stop at first failure).
# usage: bash tools/gpu_check.sh [pytest -k expression]
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s $K > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/bench.log
