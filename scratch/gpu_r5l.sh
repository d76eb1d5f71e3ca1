set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stem_fused.py -m gpu -q -x --timeout 200 --timeout-method thread -k "not resnet18" > gpurun_out/r5l.log 2>&1; rc=$?; tail -1 gpurun_out/r5l.log; [ $rc -le 1 ] || exit $rc
DMLAB_STEM_TRACE=1 timeout -k 10 120 python tools/stem_one.py --dtype u8 --iters 1 2>&1 | grep -E "trace" | tail -1
for sp in 0 5 7 9; do
  echo "split=$sp: $(DMLAB_STEM_SPLIT=$sp timeout -k 10 120 python tools/stem_one.py --dtype u8 2>&1 | tail -1)"
done
