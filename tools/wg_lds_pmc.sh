#!/bin/bash
# GPU box: LDS counters of the pp (variant 0) and tap-row (variant 46) wgrad kernels on the EDSR-L body shape
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wg_lds
for v in 0 46; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    --kernel-include-regex "wgrad_(pp|tr3)" --output-format csv -d gpurun_out/wg_lds/v$v -o pmc -- \
    python3 tools/bench_conv.py 32 $v "256,256,64,0" > gpurun_out/wg_lds/v$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for v in ('0', '46'):
    acc = collections.defaultdict(list)
    for f in glob.glob(f'gpurun_out/wg_lds/v{v}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            acc[(r['Kernel_Name'][:50], r['Counter_Name'])].append(float(r['Counter_Value']))
    for k, vals in sorted(acc.items()):
        print(v, k, round(sum(vals) / len(vals)))
PY
