set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest31.log 2>&1 && \
timeout -k 10 310 python bench.py --steps 20 --warmup 5 > gpurun_out/bench31.json 2> gpurun_out/bench31.err && \
timeout -k 10 310 python bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench31_eager.json 2> gpurun_out/bench31_eager.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof31 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --graph 0 > $GRAFT_REPO_ROOT/gpurun_out/prof31.log 2>&1
