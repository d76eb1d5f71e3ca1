# Ad-hoc GPU step (overwritten per experiment): pipelined 3x3 weight gradient (cfg 7).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/pytest_wgrad.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_wgrad.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_conv.py --batch 1024 --shapes l1_3x3,l2_3x3,l3_3x3,l4_3x3 --passes wgrad \
    --wcfgs h9,h3,w7 --iters 10 > gpurun_out/bench_wgrad_pipe.jsonl 2>> gpurun_out/bench_conv.err || exit 1
cat gpurun_out/bench_wgrad_pipe.jsonl
out=gpurun_out/bench_ab_wgrad.jsonl; : > $out
for v in "DMLAB_WGRAD_PIPE=0" "DMLAB_WGRAD_PIPE=1" "DMLAB_WGRAD_PIPE=0" "DMLAB_WGRAD_PIPE=1"; do
  echo "$v" >> $out
  env $v timeout -k 10 300 python bench.py --steps 30 --warmup 10 >> $out 2>> gpurun_out/bench_ab.err || exit 1
done
python - <<'PY'
import json
for l in open('gpurun_out/bench_ab_wgrad.jsonl'):
    l = l.strip()
    if l.startswith('{'):
        r = json.loads(l); print(r['value'], r['ms_per_step'])
    else: print(l, end=' ')
PY
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_model.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_model.log; exit $rc
