# Ad-hoc GPU step (overwritten per experiment): LeNet bwd-data padded tile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_lenet.py tests/test_graph_capture.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bd.log 2>&1 && \
for d in fp32 bf16 fp32; do timeout -k 10 300 python bench.py --model lenet --steps 300 --warmup 30 --dtype $d >> gpurun_out/lenet_bd.jsonl 2>/dev/null || exit 1; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_lenet5 -o prof -- python bench.py --model lenet --steps 40 --warmup 10 > gpurun_out/prof_lenet5.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_bd.log; cut -c1-160 gpurun_out/lenet_bd.jsonl
exit $rc
