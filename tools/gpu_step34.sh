set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest34.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --phases 5 > gpurun_out/bench34.json 2> gpurun_out/bench34.err && \
timeout -k 10 300 python bench.py --model lenet --steps 200 --warmup 20 --phases 20 > gpurun_out/bench34_lenet.json 2> gpurun_out/bench34_lenet.err && \
cd /tmp && export TMPDIR=/tmp && DMLAB_ROCTX=1 timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof34 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --graph 0 > $GRAFT_REPO_ROOT/gpurun_out/prof34.log 2>&1
