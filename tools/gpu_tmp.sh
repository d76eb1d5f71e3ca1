# Ad-hoc GPU step (overwritten per experiment): no main-stream waits for DDP hooks / shortcut join.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ns.log 2>&1 && \
for r in 1 2 3; do timeout -k 10 200 python bench.py --steps 30 --warmup 5 >> gpurun_out/bench_ns.jsonl 2>>gpurun_out/bench_ns.err || exit 1; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ns -o prof -- python bench.py --steps 7 --warmup 3 > gpurun_out/prof_ns.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_ns.log; cut -c1-170 gpurun_out/bench_ns.jsonl
exit $rc
