#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) for one kernel of a command.
# usage: bash tools/pmc_kernel.sh <tag> <kernel-regex> <command...>
TAG=$1; KRE=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" --output-format csv -d $OUT/p$i -o pmc -- "$@" > $OUT/run$i.log 2>&1 || exit 1
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(list)
waves = None
for f in sorted(glob.glob(sys.argv[1] + '/p*/pmc_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
w = sum(agg['SQ_WAVES']) / len(agg['SQ_WAVES'])
for k, v in agg.items():
    m = sum(v) / len(v)
    print(f'{k:24s} {m:14.1f}  per-wave {m / w:10.1f}')
PY
