set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest32.log 2>&1 && \
timeout -k 10 320 python bench.py --steps 20 --warmup 5 > gpurun_out/bench32.json 2> gpurun_out/bench32.err && \
timeout -k 10 320 python bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench32_eager.json 2> gpurun_out/bench32_eager.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof32 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --graph 0 > $GRAFT_REPO_ROOT/gpurun_out/prof32.log 2>&1
