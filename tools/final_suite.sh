#!/bin/bash
# Closing evidence: the whole GPU test suite, smoke(), and the bench line of every workload (default
# configuration, as the driver runs it): bash tools/final_suite.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gpu_tests.log 2>&1; rc=$?; tail -4 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 \
  && tail -2 $OUT/smoke.log || { tail -20 $OUT/smoke.log; exit 1; }
for wl in edsr rcan swinir rrdb; do
  timeout -k 10 400 python -u bench.py --workload $wl > $OUT/bench_$wl.log 2>&1 || { tail -20 $OUT/bench_$wl.log; exit 1; }
  grep '^{"metric' $OUT/bench_$wl.log > $OUT/bench_$wl.json
  python3 -c "import json; d=json.load(open('$OUT/bench_$wl.json')); r=d['roofline']; print('$wl', d['ms_per_step'], d['value'], r['kernel'], r['frac'], d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"
done
