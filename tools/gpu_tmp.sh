# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=s5h
timeout -k 10 300 python -u -m pytest tests/test_native_lenet.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$t.log 2>&1 || { tail -40 gpurun_out/pytest_$t.log; exit 1; }
tail -4 gpurun_out/pytest_$t.log
