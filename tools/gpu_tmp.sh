# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${1:-xcd}
DMLAB_HALO_XCD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_resnet_kernels.py -m gpu -k "halo or fwd or dgrad or prebn" > gpurun_out/test_${t}.log 2>&1 && tail -2 gpurun_out/test_${t}.log || { tail -40 gpurun_out/test_${t}.log; exit 1; }
for x in 0 1 0 1; do
  DMLAB_HALO_XCD=$x timeout -k 10 200 python tools/bench_conv.py --batch 512 --iters 30 --cfgs 39,41,42,44 --passes fwd,dgrad --shapes l1_3x3,l2_3x3,l3_3x3,l4_3x3 > gpurun_out/hx_$x.jsonl 2>gpurun_out/hx_$x.err || exit 1
  python -c "
import json
for l in open('gpurun_out/hx_$x.jsonl'):
    r = json.loads(l); print('xcd $x', r['shape'], {k: v for k, v in r.items() if k.endswith('_TF')})"
done
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 80 --warmup 10 > gpurun_out/b_${t}.json 2>gpurun_out/b_${t}.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/b_${t}.json')); print('$tag', d['value'], d['ms_per_step'])" | tee -a gpurun_out/bench_$t.txt
}
for r in 1 2; do
  run xcd0 DMLAB_HALO_XCD=0
  run xcd1 DMLAB_HALO_XCD=1
done
