set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -m gpu -q -k "bn_reduce" --timeout 120 --timeout-method thread > gpurun_out/r5ad_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5ad_tests.log; [ $rc -le 1 ] || exit $rc
for f in 1 0 1 0 1 0 1 0; do
  echo "ypre=$f $(DMLAB_HALO_YPRE=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d.get("final_loss"))')" || exit 1
done
export AMD_SERIALIZE_KERNEL=3
for f in 1 0; do
DMLAB_HALO_YPRE=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5ad_$f -o p -- python bench.py --steps 4 --warmup 2 --phases 0 > gpurun_out/r5ad_prof$f.log 2>&1; echo "prof$f rc=$?"
f2=$(find gpurun_out/prof_r5ad_$f -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py "$f2" 6 > gpurun_out/r5ad_profsum$f.txt 2>&1
grep conv_halo gpurun_out/r5ad_profsum$f.txt
done
