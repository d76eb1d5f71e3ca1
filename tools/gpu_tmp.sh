# Ad-hoc GPU step (overwritten per experiment): native vs stock-torch loss at large per-GPU batch.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/batch_numerics.jsonl; : > $out
for b in 512 1024; do
  for be in native torch; do
    for s in 1 4; do
      timeout -k 10 240 python bench.py --batch $b --backend $be --steps $s --warmup 0 >> $out 2>> gpurun_out/batch_numerics.err || { tail -5 gpurun_out/batch_numerics.err; exit 1; }
    done
  done
done
python -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['config']['per_gpu_batch'], d['config']['backend'], d['steps'], d['final_loss'])
"
