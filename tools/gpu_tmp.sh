# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=s4o
timeout -k 10 400 python -u -m pytest tests/test_native_resnet_model.py tests/test_native_resnet_kernels.py tests/test_graph_capture.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$t.log 2>&1 || { tail -40 gpurun_out/pytest_$t.log; exit 1; }
tail -1 gpurun_out/pytest_$t.log
for r in 1 2 3; do
timeout -k 10 200 python bench.py --steps 30 --warmup 5 2>> gpurun_out/bench_$t.err | cut -c 80-130 || exit 1
done
