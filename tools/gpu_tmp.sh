# Ad-hoc GPU step (overwritten per experiment): next-batch input packing prefetch A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pf.log 2>&1 && \
for r in 1 2 3; do for e in 0 1; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --prefetch $e > gpurun_out/b.json 2>>gpurun_out/bench_ab.err || exit 1
  echo "prefetch=$e $(cut -c1-170 gpurun_out/b.json)" >> gpurun_out/pf_ab.txt
done; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_pf -o prof -- python bench.py --steps 7 --warmup 3 > gpurun_out/prof_pf.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_pf.log; cat gpurun_out/pf_ab.txt
exit $rc
