# Ad-hoc GPU step (overwritten per experiment): fp32 GEMM split-K (LeNet).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_lenet.py tests/test_graph_capture.py tests/test_optim_kernels.py tests/test_multiproc_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sk.log 2>&1 && \
for d in fp32 bf16 fp32 bf16; do timeout -k 10 300 python bench.py --model lenet --steps 300 --warmup 30 --dtype $d >> gpurun_out/lenet_sk.jsonl 2>/dev/null || exit 1; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_lenet4 -o prof -- python bench.py --model lenet --steps 40 --warmup 10 > gpurun_out/prof_lenet4.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_sk.log; cut -c1-160 gpurun_out/lenet_sk.jsonl
exit $rc
