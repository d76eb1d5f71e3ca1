# Ad-hoc GPU step (overwritten per experiment): wgrad cfg 8 tests, micro-bench, A/B.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad_res64" \
    > gpurun_out/pytest_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_$tag.log; exit 1; }
timeout -k 10 200 python tools/bench_conv.py --batch 1024 --shapes l1_3x3 --passes wgrad --wcfgs h3,q8 \
    > gpurun_out/bench_conv_$tag.jsonl 2> gpurun_out/bench_conv_$tag.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
tail -3 gpurun_out/pytest_$tag.log; cat gpurun_out/bench_conv_$tag.jsonl; cut -c1-200 gpurun_out/bench_$tag.json
