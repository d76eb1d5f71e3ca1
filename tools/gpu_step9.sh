set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -q -x > gpurun_out/pytest9.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench9.json 2> gpurun_out/bench9.err
