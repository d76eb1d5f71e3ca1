# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=s4e
timeout -k 10 400 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$t.log 2>&1 || { tail -30 gpurun_out/pytest_$t.log; exit 1; }
tail -2 gpurun_out/pytest_$t.log
b() { timeout -k 10 200 python bench.py --steps 30 --warmup 5 "$@" 2>> gpurun_out/bench_$t.err | cut -c 80-118; }
for r in 1 2; do
echo "eager side";   b --graph 0 || exit 1
echo "eager noside"; DMLAB_WGRAD_STREAM=0 b --graph 0 || exit 1
echo "graph noside"; DMLAB_WGRAD_STREAM=0 b || exit 1
echo "graph side"; b || exit 1
echo "graph side256"; DMLAB_WGRAD_STREAM_MIN_COUT=256 b || exit 1
echo "eager side256"; DMLAB_WGRAD_STREAM_MIN_COUT=256 b --graph 0 || exit 1
done
