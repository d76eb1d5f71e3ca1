# Ad-hoc GPU step (overwritten per experiment): stock PyTorch-ROCm ResNet-18 at 1024 per GPU.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/probe_stock.py --resnet-batches 1024 > gpurun_out/stock_b1024.jsonl 2> gpurun_out/stock_b1024.err
rc=$?
cat gpurun_out/stock_b1024.jsonl | cut -c1-200
exit $rc
