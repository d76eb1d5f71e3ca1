# Ad-hoc GPU step (overwritten per experiment): CU-masked weight-gradient stream A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/cumask_ab.jsonl; : > $out
for m in "" 77777777 7f7f7f7f "" 3f3f3f3f 77777777 7f7f7f7f; do
  echo "mask=$m" >> $out
  DMLAB_WGRAD_CUMASK=$m timeout -k 10 200 python bench.py --steps 40 --warmup 8 >> $out 2>> gpurun_out/cumask_ab.err || exit 1
done
cat $out | cut -c1-200
