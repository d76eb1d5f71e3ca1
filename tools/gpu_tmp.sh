# Ad-hoc GPU step (overwritten per experiment): res64 layer-1 conv tests, micro-bench, A/B.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "res64" \
    > gpurun_out/pytest_$tag.log 2>&1 && \
timeout -k 10 200 python tools/bench_conv.py --batch 1024 --shapes l1_3x3 --cfgs 39,41,80 --passes fwd,dgrad --pre \
    > gpurun_out/bench_conv_$tag.jsonl 2> gpurun_out/bench_conv_$tag.err && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err && \
DMLAB_NO_RES64=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_nores_$tag.json 2> gpurun_out/bench_nores_$tag.err && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_$tag.json 2>> gpurun_out/bench_$tag.err
rc=$?
tail -3 gpurun_out/pytest_$tag.log; cat gpurun_out/bench_conv_$tag.jsonl; cut -c1-200 gpurun_out/bench_$tag.json gpurun_out/bench_nores_$tag.json
exit $rc
