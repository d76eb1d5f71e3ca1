# Ad-hoc GPU step (overwritten per experiment): persistent stem conv A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -k "stem or resnet18 or prefetch" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_stem.log 2>&1 && \
for e in 0 1 0 1; do
  echo "persist=$e $(DMLAB_STEM_PERSIST=$e timeout -k 10 120 python tools/bench_conv.py --batch 512 --cfgs 60 --passes fwd --shapes stem_s2d 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> gpurun_out/stem_ab.txt || exit 1
done && \
for r in 1 2 3; do for e in 0 1; do
  DMLAB_STEM_PERSIST=$e timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/b.json 2>>gpurun_out/bench_ab.err || exit 1
  echo "persist=$e $(cut -c1-170 gpurun_out/b.json)" >> gpurun_out/stem_ab.txt
done; done
rc=$?
tail -2 gpurun_out/pytest_stem.log; cat gpurun_out/stem_ab.txt
exit $rc
