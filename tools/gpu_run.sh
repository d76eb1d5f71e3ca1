# Standard GPU-box check: GPU test suite, headline bench, per-kernel rocprof stats.
#   gpurun --timeout 1100 -- bash tools/gpu_run.sh <tag>
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o prof -- \
    python bench.py --steps 7 --warmup 3 --graph 0 > gpurun_out/prof_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$tag.log; cat gpurun_out/bench_$tag.json
exit $rc
