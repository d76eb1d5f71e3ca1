# Ad-hoc GPU step (overwritten per experiment): ResNet eager vs hipGraph re-check.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do for gph in 0 1; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --graph $gph > gpurun_out/b.json 2>>gpurun_out/bench_graph.err || exit 1
  echo "graph=$gph $(cut -c1-170 gpurun_out/b.json)" >> gpurun_out/graph_ab.txt
done; done
cat gpurun_out/graph_ab.txt
