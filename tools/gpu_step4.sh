set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_native_resnet_model.py -q -x > gpurun_out/pytest4.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_r18.json 2> gpurun_out/bench_r18.err && \
timeout -k 10 300 python bench.py --model lenet --steps 200 --warmup 20 > gpurun_out/bench_lenet.json 2> gpurun_out/bench_lenet.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r18 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
