#!/bin/bash
# Selected GPU tests on the box: bash tools/gpu_tests.sh <tag> <pytest args...>
# -> gpurun_out/<tag>/tests.log (one process, per-test thread timeout)
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest "$@" -m gpu -v -s --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|rel err|worst|passed|failed" $OUT/tests.log | tail -60
exit $rc
