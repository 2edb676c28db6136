#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py -k "halo_vs or ring" > gpurun_out/ringtest.log 2>&1
rc=$?; echo rc=$rc; tail -3 gpurun_out/ringtest.log; exit $rc
