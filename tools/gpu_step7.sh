set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_native_resnet_kernels.py -q -x > gpurun_out/pytest7.log 2>&1 && \
timeout -k 10 600 python tools/bench_conv.py > gpurun_out/conv7.jsonl 2> gpurun_out/conv7.err
