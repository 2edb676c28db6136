#!/bin/bash
# GPU box: per-step kernel tables of libA vs libB (rocprofv3 kernel trace, eager steps).
# usage: W=swinir bash tools/kt_ab.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in A B; do
  rm -rf gpurun_out/kt_$v
  SR_HIP_LIB=tools/ab/lib$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_$v -o kt -- \
    python3 -u bench.py --workload ${W:-swinir} --steps 3 --warmup 1 --no-cpu-baseline --no-trace --graph 0 \
    > gpurun_out/kt_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/kt_$v -name '*kernel_trace.csv' | head -1)
  echo "== $v"; python3 tools/step_kernels.py "$f" ${TOP:-14}
done
