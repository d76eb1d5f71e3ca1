# Ad-hoc GPU step (overwritten per experiment): single-block CE.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_lenet.py tests/test_graph_capture.py tests/test_tasks_cpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ce.log 2>&1 && \
for d in fp32 bf16 fp32 bf16; do timeout -k 10 300 python bench.py --model lenet --steps 300 --warmup 30 --dtype $d >> gpurun_out/lenet_ce.jsonl 2>/dev/null || exit 1; done
rc=$?
tail -2 gpurun_out/pytest_ce.log; cut -c1-160 gpurun_out/lenet_ce.jsonl
exit $rc
