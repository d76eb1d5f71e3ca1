set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_q9.log 2>&1 && \
DMLAB_FUSE_BN_BWD=1 timeout -k 10 300 python -u -m pytest tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread >> gpurun_out/pytest_q9.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_q9.json 2> gpurun_out/bench_q9.err && \
DMLAB_FUSE_BN_BWD=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_q9f.json 2> gpurun_out/bench_q9f.err
rc=$?; grep passed gpurun_out/pytest_q9.log; cat gpurun_out/bench_q9.json gpurun_out/bench_q9f.json | cut -c1-140; exit $rc
