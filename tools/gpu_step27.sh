#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_native_resnet_kernels.py -x -q -k "conv_fwd or dgrad" > gpurun_out/t27.log 2>&1 &&
timeout -k 10 300 python tools/bench_conv.py --passes fwd,dgrad --iters 30 --cfgs 12,20,38,37,39 > gpurun_out/bc27.jsonl 2>&1
