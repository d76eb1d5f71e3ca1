#!/bin/bash
# conv kernel variants: numerics + micro-bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_native_resnet_kernels.py -x -q > gpurun_out/t13.log 2>&1 &&
timeout -k 10 300 python tools/bench_conv.py --passes fwd,dgrad --iters 30 --cfgs 12,15,16,20,21,24,25 > gpurun_out/bc13.jsonl 2>&1
