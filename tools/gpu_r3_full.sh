# full GPU test suite + smoke (what the driver runs at round end)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_full
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3_full/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r3_full/pytest.log)"
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_full/smoke.log 2>&1
echo "smoke rc=$? $(tail -1 gpurun_out/r3_full/smoke.log)"
