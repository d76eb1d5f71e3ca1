# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=s4f
timeout -k 10 500 python -u -m pytest tests/test_multiproc_gpu.py tests/test_native_resnet_kernels.py -k "ddp_resnet or s2d" -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_$t.log 2>&1 || { tail -40 gpurun_out/pytest_$t.log; exit 1; }
tail -2 gpurun_out/pytest_$t.log
timeout -k 10 300 python tools/bench_conv.py --shapes stem_s2d --cfgs 13,16,17,11,14,35 --passes fwd,wgrad --wcfgs v2 --batch 512 > gpurun_out/conv_$t.jsonl 2>&1 || exit 1
grep shape gpurun_out/conv_$t.jsonl
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_$t.json 2> gpurun_out/bench_$t.err || exit 1
cut -c 1-200 gpurun_out/bench_$t.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$t -o prof -- \
    python bench.py --steps 5 --warmup 3 > gpurun_out/prof_$t.log 2>&1
