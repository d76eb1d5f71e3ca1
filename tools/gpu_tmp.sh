# Ad-hoc GPU step (overwritten per experiment): per-channel-group one-launch BN finalize A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -k "finalize or fused_bn_backward or bn_forward or model or resnet" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fin.log 2>&1 && \
DMLAB_FUSED_FIN=1 timeout -k 10 300 python -u -m pytest tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fin_model.log 2>&1 && \
for r in 1 2 3; do for e in 0 1; do
  DMLAB_FUSED_FIN=$e timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/b.json 2>>gpurun_out/bench_ab.err || exit 1
  echo "fused_fin=$e $(cut -c1-170 gpurun_out/b.json)" >> gpurun_out/fin_ab.txt
done; done
rc=$?
tail -2 gpurun_out/pytest_fin.log; tail -2 gpurun_out/pytest_fin_model.log; cat gpurun_out/fin_ab.txt
exit $rc
