set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stem_fused.py -m gpu -q -x --timeout 200 --timeout-method thread -k "not resnet18" > gpurun_out/r5i_stem.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5i_stem.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for sp in 0 5 7 9; do
  echo "split=$sp: $(DMLAB_STEM_SPLIT=$sp timeout -k 10 120 python tools/stem_one.py --dtype u8 2>&1 | tail -1)"
done
for ab in 1 4 5; do
  echo "ablate=$ab: $(DMLAB_STEM_ABLATE=$ab timeout -k 10 120 python tools/stem_one.py --dtype u8 2>&1 | tail -1)"
done
