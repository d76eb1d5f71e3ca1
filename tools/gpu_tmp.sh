# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=s4b
for b in 384 768 1024; do
  timeout -k 10 200 python bench.py --steps 15 --warmup 3 --batch $b > gpurun_out/bench_${t}_b$b.json 2>> gpurun_out/bench_$t.err || exit $?
done
timeout -k 10 300 python tools/probe_stock.py --resnet-batches 512 > gpurun_out/stock_$t.jsonl 2>> gpurun_out/bench_$t.err
rc=$?
cat gpurun_out/bench_${t}_*.json gpurun_out/stock_$t.jsonl | cut -c 1-260
exit $rc
