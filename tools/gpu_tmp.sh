# Ad-hoc GPU step (overwritten per experiment): weight-gradient m-split target at 1024 img/GPU.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/wgrad_blocks_b1024.jsonl; : > $out
for b in 512 1024 768 512 1024 768; do
  echo "blocks=$b" >> $out
  DMLAB_WGRAD_BLOCKS=$b timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> $out 2>> gpurun_out/wgrad_blocks_b1024.err || exit 1
done
cut -c60-110 $out
