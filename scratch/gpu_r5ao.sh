set -o pipefail
export TMPDIR=/tmp
DMLAB_BN_LEAN=1 timeout -k 10 600 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -m gpu -q -k "bn or resnet18" --timeout 300 --timeout-method thread > gpurun_out/r5ao_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5ao_tests.log; [ $rc -le 1 ] || exit $rc
for f in 1 0 1 0 1 0 1 0; do
  echo "lean=$f $(DMLAB_BN_LEAN=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d.get("param_checksum"))')" || exit 1
done
DMLAB_BN_LEAN=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r5ao -o k -- python bench.py --steps 6 --warmup 3 --phases 0 > gpurun_out/r5ao_kt.log 2>&1; echo "kt rc=$?"
f=$(find gpurun_out/prof_r5ao -name "*kernel_trace.csv" | head -1); python tools/step_trace.py "$f" > gpurun_out/r5ao_step.txt 2>&1; echo "steptrace rc=$?"; tail -1 gpurun_out/r5ao_step.txt
