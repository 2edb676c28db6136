#!/bin/bash
# GPU box: effective clock of the EDSR-L body kernels (MI355X_MICROARCH.md "DVFS give-back": GRBM_GUI_ACTIVE / 8 /
# kernel time) with SQ_INSTS_MFMA, from the conv microbench at B 32 (pph fwd / dgrad, pp wgrad)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/clk
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_BUSY_CYCLES --kernel-trace --kernel-include-regex "pph|wgrad_pp" \
  --output-format csv -d gpurun_out/clk -o clk -- python3 tools/bench_conv.py 32 0 "256,256,64,0" > gpurun_out/clk/run.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/clk/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        cnt[r['Kernel_Name'][:60]][r['Counter_Name']].append(float(r['Counter_Value']))
        if 'Start_Timestamp' in r:
            cnt[r['Kernel_Name'][:60]]['dur_ns'].append(float(r['End_Timestamp']) - float(r['Start_Timestamp']))
for k, d in cnt.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
