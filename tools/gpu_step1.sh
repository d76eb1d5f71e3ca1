set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_optim_kernels.py -x -q > gpurun_out/pytest1.log 2>&1 && \
timeout -k 10 600 python tools/probe_stock.py > gpurun_out/stock.jsonl 2> gpurun_out/stock.err
