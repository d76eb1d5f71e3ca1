set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_native_resnet_model.py tests/test_stem_fused.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5ak_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5ak_tests.log; [ $rc -le 1 ] || exit $rc
for f in 1 0 1 0 1 0 1 0; do
  echo "packaux=$f $(DMLAB_PACK_AUX=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d.get("final_loss"), d.get("param_checksum"))')" || exit 1
done
