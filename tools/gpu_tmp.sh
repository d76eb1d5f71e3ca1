# Ad-hoc GPU step (overwritten per experiment): native TP head test + stride-2 tile/split sweep.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_native_lenet.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_$tag.log; exit 1; }
timeout -k 10 300 python tools/bench_conv.py --batch 1024 --shapes l2_3x3s2 --cfgs 15,16,12,13,10,17,91,92,93 --passes fwd,dgrad \
    > gpurun_out/bench_conv_$tag.jsonl 2> gpurun_out/bench_conv_$tag.err || exit 1
timeout -k 10 300 python tools/bench_conv.py --batch 1024 --shapes l2_3x3s2,l2_down --passes wgrad --wcfgs g2,g3,w6 --smul 0.5,1,2,4 \
    >> gpurun_out/bench_conv_$tag.jsonl 2>> gpurun_out/bench_conv_$tag.err || exit 1
tail -3 gpurun_out/pytest_$tag.log; cat gpurun_out/bench_conv_$tag.jsonl
