#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/gemm_ceiling.py > gpurun_out/gemm_ceiling.jsonl 2>&1 &&
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
