set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_stem_fused.py -m gpu -q -x --timeout 200 --timeout-method thread -k "not resnet18" > gpurun_out/r5g_stem.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5g_stem.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for ab in 0 1 2 3 4 5 7 12 15; do
  echo "ablate=$ab: $(DMLAB_STEM_ABLATE=$ab timeout -k 10 120 python tools/stem_one.py --dtype u8 2>&1 | tail -1)"
done
