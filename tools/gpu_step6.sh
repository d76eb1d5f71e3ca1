set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_conv.py > gpurun_out/conv6.jsonl 2> gpurun_out/conv6.err
