#!/bin/bash
# GPU box: parity tests, smoke, bench (each step under its own time limit; stop at first failure).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
tail -3 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/bench.log
