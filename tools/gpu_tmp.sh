# Ad-hoc GPU step (overwritten per experiment): res64 v3 vs v1 tests, micro-bench, A/B.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "res64" \
    > gpurun_out/pytest_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_$tag.log; exit 1; }
for v in 3 1 3; do
DMLAB_RES64_V=$v timeout -k 10 200 python tools/bench_conv.py --batch 1024 --shapes l1_3x3 --cfgs 80 --passes fwd,dgrad --pre \
    >> gpurun_out/bench_conv_$tag.jsonl 2>> gpurun_out/bench_conv_$tag.err || exit 1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
DMLAB_RES64_V=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_v1_$tag.json 2> gpurun_out/bench_v1_$tag.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
tail -3 gpurun_out/pytest_$tag.log; cat gpurun_out/bench_conv_$tag.jsonl; cut -c1-200 gpurun_out/bench_$tag.json gpurun_out/bench_v1_$tag.json
