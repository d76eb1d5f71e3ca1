# Ad-hoc GPU step (overwritten per experiment): persistent single-chunk halo conv A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -k "halo or prebn or resnet18 or tail or dgrad" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_hp.log 2>&1 && \
for e in 0 1 0 1; do
  echo "pers=$e $(DMLAB_HALO_PERS=$e timeout -k 10 120 python tools/bench_conv.py --batch 512 --cfgs 39 --passes fwd,dgrad --shapes l1_3x3 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> gpurun_out/hp_ab.txt || exit 1
done && \
for r in 1 2 3; do for e in 0 1; do
  DMLAB_HALO_PERS=$e timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/b.json 2>>gpurun_out/bench_ab.err || exit 1
  echo "pers=$e $(cut -c1-170 gpurun_out/b.json)" >> gpurun_out/hp_ab.txt
done; done
rc=$?
tail -2 gpurun_out/pytest_hp.log; cat gpurun_out/hp_ab.txt
exit $rc
