# Ad-hoc GPU step (overwritten per experiment): persistent halo opt-in test.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -k "persistent_opt_in or bn_backward_apply_on_load" -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_po.log 2>&1
rc=$?
tail -12 gpurun_out/pytest_po.log
exit $rc
