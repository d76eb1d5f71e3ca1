#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_conv.py --passes fwd --iters 30 --shapes gemm_k2048_n256,gemm_k1024_n512,l3_3x3  > gpurun_out/bc17.jsonl 2>&1 &&
timeout -k 10 200 python tools/gemm_ceiling.py > gpurun_out/gc17.jsonl 2>&1
