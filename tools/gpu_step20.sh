#!/bin/bash
set -o pipefail
mkdir -p gpurun_out

timeout -k 10 300 python tools/bench_conv.py --passes wgrad --iters 20 --wcfgs v2,h9,h3 > gpurun_out/bc20.jsonl 2>&1
