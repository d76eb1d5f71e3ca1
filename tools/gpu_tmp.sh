# Ad-hoc GPU step (overwritten per experiment): colsum batching check.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_lenet.py tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cs.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_cs -o prof -- python bench.py --steps 7 --warmup 3 > gpurun_out/prof_cs.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_cs.log
exit $rc
