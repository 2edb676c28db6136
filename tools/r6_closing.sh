#!/bin/bash
# Round-6 closing evidence, part 1: the whole GPU suite, smoke(), and the default bench line (the
# driver's command: EDSR headline + per-workload sub-records) -> gpurun_out/<tag>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gpu_tests.log 2>&1; rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 \
  && tail -2 $OUT/smoke.log || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 780 python -u bench.py > $OUT/bench_suite.log 2> $OUT/bench_suite.err || { tail -20 $OUT/bench_suite.err; exit 1; }
grep '^{"metric' $OUT/bench_suite.log > $OUT/bench_suite.json
python3 -c "
import json; d=json.load(open('$OUT/bench_suite.json'))
print('edsr', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])
for k, s in d.get('sub_records', {}).items():
    print(k, s.get('ms_per_step'), s.get('value'), s['roofline']['kernel'] if s.get('roofline') else None, s['roofline']['frac'] if s.get('roofline') else None)
"
