# Ad-hoc GPU step (overwritten per experiment): layer-1 halo conv launch-bounds A/B
# (alt/_C_minb2.so = the extension built with -DDM_HALO39_MINB=2).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
so=dmlab/_C.cpython-310-x86_64-linux-gnu.so
cp $so alt/_C_default.so
out=gpurun_out/minb_ab.jsonl; : > $out
for v in default minb2 default minb2 default minb2; do
  cp alt/_C_$v.so $so
  echo "variant=$v" >> $out
  timeout -k 10 200 python bench.py --steps 40 --warmup 8 >> $out 2>> gpurun_out/minb_ab.err || exit 1
done
cp alt/_C_minb2.so $so
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k halo > gpurun_out/pytest_minb.log 2>&1 || { tail -20 gpurun_out/pytest_minb.log; exit 1; }
tail -1 gpurun_out/pytest_minb.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_minb2 -o prof -- python bench.py --steps 7 --warmup 3 > gpurun_out/prof_minb2.log 2>&1
cp alt/_C_default.so $so
cut -c1-120 $out
