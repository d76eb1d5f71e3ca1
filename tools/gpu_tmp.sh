# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=s5i
timeout -k 10 900 python -u tools/probe_stock.py --tuned --resnet-batches 512 2> gpurun_out/stock_$t.err | tee gpurun_out/stock_tuned_$t.jsonl || { tail -20 gpurun_out/stock_$t.err; exit 1; }
