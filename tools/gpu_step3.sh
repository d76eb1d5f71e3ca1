set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -q -x > gpurun_out/pytest3.log 2>&1
