# Ad-hoc GPU step (overwritten per experiment): BN-backward apply on load (layer-1 c1) A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bol.log 2>&1 && \
for r in 1 2 3; do for e in 0 1; do
  DMLAB_BN_BWD_ON_LOAD=$e timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/b.json 2>>gpurun_out/bench_ab.err || exit 1
  echo "on_load=$e $(cut -c1-170 gpurun_out/b.json)" >> gpurun_out/bol_ab.txt
done; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_bol -o prof -- python bench.py --steps 7 --warmup 3 > gpurun_out/prof_bol.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_bol.log; cat gpurun_out/bol_ab.txt
exit $rc
