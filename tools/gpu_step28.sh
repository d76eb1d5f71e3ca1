#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_multiproc_gpu.py tests/test_native_lenet.py -x -q -k "xgmi or lowp" > gpurun_out/t28.log 2>&1
