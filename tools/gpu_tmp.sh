# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=s5c
timeout -k 10 500 python -u -m pytest tests/test_multiproc_gpu.py -k "xgmi" -m gpu -x -v --timeout 280 --timeout-method thread \
    > gpurun_out/pytest_$t.log 2>&1 || { tail -60 gpurun_out/pytest_$t.log; exit 1; }
tail -15 gpurun_out/pytest_$t.log
