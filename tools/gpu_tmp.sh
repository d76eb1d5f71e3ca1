# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=s5a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$t.log 2>&1 || { tail -40 gpurun_out/pytest_$t.log; exit 1; }
tail -1 gpurun_out/pytest_$t.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$t.log 2>&1 || { tail -20 gpurun_out/smoke_$t.log; exit 1; }
timeout -k 10 200 python bench.py 2>> gpurun_out/bench_$t.err | tee gpurun_out/bench_$t.json || exit 1
