# Ad-hoc GPU step (overwritten per experiment): weight-gradient m-split target A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/wgrad_blocks_ab.jsonl; : > $out
for b in 512 256 1024 384 512 768 256 1024; do
  echo "blocks=$b" >> $out
  DMLAB_WGRAD_BLOCKS=$b timeout -k 10 200 python bench.py --steps 40 --warmup 8 >> $out 2>> gpurun_out/wgrad_blocks_ab.err || exit 1
done
cut -c1-120 $out
