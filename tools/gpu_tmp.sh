# Ad-hoc GPU step (overwritten per experiment): fused identity skip tests + A/B on one box.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread -k "masked_add or model or resnet" \
    > gpurun_out/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_$tag.log; exit 1; }
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
DMLAB_NO_FUSED_SKIP=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_nofs_$tag.json 2>> gpurun_out/bench_nofs_$tag.err || exit 1
done
tail -3 gpurun_out/pytest_$tag.log; cut -c1-200 gpurun_out/bench_$tag.json gpurun_out/bench_nofs_$tag.json
