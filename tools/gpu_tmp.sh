# Ad-hoc GPU step (overwritten per experiment): fused LeNet step tests + bench; step-time diagnostics.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_lenet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lenet.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_lenet.log
[ $rc -ne 0 ] && exit $rc
out=gpurun_out/bench_lenet_fused.jsonl; : > $out
for f in 1 0 1 0; do
  echo "fused=$f" >> $out
  timeout -k 10 200 python bench.py --model lenet --fused $f --steps 500 --warmup 50 >> $out 2>> gpurun_out/bench_lenet.err || exit 1
done
echo "fused=1 bf16" >> $out
timeout -k 10 200 python bench.py --model lenet --dtype bf16 --steps 500 --warmup 50 >> $out 2>> gpurun_out/bench_lenet.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lenet -o prof -- \
    python bench.py --model lenet --steps 50 --warmup 10 > gpurun_out/prof_lenet.log 2>&1 || exit 1
out2=gpurun_out/bench_diag.jsonl; : > $out2
for v in "X=0" "DMLAB_DIAG_SKIP_WGRAD=1" "DMLAB_NO_PIPE=1" "DMLAB_WGRAD_STREAM=0"; do
  echo "$v" >> $out2
  env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> $out2 2>> gpurun_out/bench_diag.err || exit 1
done
python - <<'PY'
import json
for f in ('gpurun_out/bench_lenet_fused.jsonl','gpurun_out/bench_diag.jsonl'):
    for l in open(f):
        l=l.strip()
        if l.startswith('{'):
            r=json.loads(l); print(r['value'], r['ms_per_step'], r['config'].get('hip_graph'))
        else: print(l, end=' ')
PY
