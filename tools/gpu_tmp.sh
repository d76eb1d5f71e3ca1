# Ad-hoc GPU step (overwritten per experiment): single-band halo epilogue A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_native_resnet_kernels.py -k "halo or tail_split or prebn or fused_bn_backward or dgrad" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_epi.log 2>&1 && \
for e in 1 0 1 0; do
  echo "bands=$e $(DMLAB_EPI_BANDS=$e timeout -k 10 120 python tools/bench_conv.py --batch 512 --cfgs 39,41 --passes fwd,dgrad --shapes l1_3x3,l3_3x3,l4_3x3 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')" >> gpurun_out/epi_ab.txt || exit 1
done && \
for r in 1 2; do for e in 1 0; do
  DMLAB_EPI_BANDS=$e timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/b.json 2>>gpurun_out/bench_ab.err || exit 1
  echo "bands=$e $(cut -c1-170 gpurun_out/b.json)" >> gpurun_out/epi_ab.txt
done; done
rc=$?
tail -2 gpurun_out/pytest_epi.log; cat gpurun_out/epi_ab.txt
exit $rc
