# Ad-hoc GPU step (overwritten per experiment): halo-pipe kernel tests, pruned kernel set,
# fused LeNet v2, ResNet A/B, multi-rank tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -x -q --timeout 120 --timeout-method thread -k hpipe > gpurun_out/pytest_hpipe.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_hpipe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py tests/test_native_lenet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_prune.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_prune.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/bench_ab_hpipe.jsonl; : > $out
for v in 0 1 0 1; do
  echo "NO_HPIPE=$v" >> $out
  DMLAB_NO_HPIPE=$v timeout -k 10 300 python bench.py --steps 30 --warmup 10 >> $out 2>> gpurun_out/bench_ab.err || exit 1
done
out2=gpurun_out/bench_lenet_fused2.jsonl; : > $out2
for f in 1 0; do
  echo "fused=$f" >> $out2
  timeout -k 10 200 python bench.py --model lenet --fused $f --steps 500 --warmup 50 >> $out2 2>> gpurun_out/bench_lenet.err || exit 1
done
echo "fused=1 bf16" >> $out2
timeout -k 10 200 python bench.py --model lenet --fused 1 --dtype bf16 --steps 500 --warmup 50 >> $out2 2>> gpurun_out/bench_lenet.err || exit 1
python - <<'PY'
import json
for fn in ('gpurun_out/bench_ab_hpipe.jsonl', 'gpurun_out/bench_lenet_fused2.jsonl'):
    for l in open(fn):
        l=l.strip()
        if l.startswith('{'):
            r=json.loads(l); print(r['value'], r['ms_per_step'], r['config'].get('hip_graph'))
        else: print(l, end=' ')
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3b -o prof -- \
    python bench.py --steps 10 --warmup 5 > gpurun_out/prof_r3b.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lenet2 -o prof -- \
    python bench.py --model lenet --fused 1 --steps 50 --warmup 10 > gpurun_out/prof_lenet2.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_multiproc_gpu.py -x -v --timeout 280 --timeout-method thread -k "lenet_fused or ddp_xgmi_graph or pipeline_xgmi or bench_lenet" > gpurun_out/pytest_mp.log 2>&1
rc=$?; tail -12 gpurun_out/pytest_mp.log; exit $rc
