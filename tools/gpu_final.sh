# Round-end style check on one MI355X: full GPU tests, smoke, headline bench, per-kernel stats.
#   gpurun --timeout 1100 -- bash tools/gpu_final.sh <tag>
set -o pipefail
tag=${1:-final}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default_$tag.json 2> gpurun_out/bench_default_$tag.err && \
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err && \
timeout -k 10 300 python bench.py --model lenet --steps 200 --warmup 20 > gpurun_out/bench_lenet_$tag.json 2> gpurun_out/bench_lenet_$tag.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o prof -- \
    python bench.py --steps 7 --warmup 3 > gpurun_out/prof_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$tag.log; tail -1 gpurun_out/smoke_$tag.log; cat gpurun_out/bench_default_$tag.json gpurun_out/bench_$tag.json gpurun_out/bench_lenet_$tag.json
exit $rc
