# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${1:-wxcd2}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_resnet_kernels.py -m gpu -k "wgrad" > gpurun_out/test_${t}.log 2>&1 && tail -2 gpurun_out/test_${t}.log || { tail -40 gpurun_out/test_${t}.log; exit 1; }
for x in 0 1 0 1; do
  DMLAB_WGRAD_XCD=$x timeout -k 10 200 python tools/bench_conv.py --batch 512 --iters 30 --wcfgs h9,h3 --passes wgrad --shapes l1_3x3,l2_3x3,l3_3x3,l4_3x3 > gpurun_out/wx_$x.jsonl 2>gpurun_out/wx_$x.err || exit 1
  python -c "
import json
for l in open('gpurun_out/wx_$x.jsonl'):
    r = json.loads(l); print('wxcd $x', r['shape'], {k: v for k, v in r.items() if k.endswith('_TF')})"
done
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 80 --warmup 10 > gpurun_out/b_${t}.json 2>gpurun_out/b_${t}.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/b_${t}.json')); print('$tag', d['value'], d['ms_per_step'])" | tee -a gpurun_out/bench_$t.txt
}
for r in 1 2; do
  run wx0 DMLAB_WGRAD_XCD=0
  run wx1 DMLAB_WGRAD_XCD=1
done
