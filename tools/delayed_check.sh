cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/det
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_train_step_gpu.py -k delayed > gpurun_out/det/delayed.log 2>&1; echo "delayed rc=$? $(tail -1 gpurun_out/det/delayed.log)"
