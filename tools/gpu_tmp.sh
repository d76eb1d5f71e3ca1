# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${1:-ws7}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_resnet_model.py -m gpu -k "stem" > gpurun_out/test_${t}.log 2>&1 && tail -2 gpurun_out/test_${t}.log || { tail -40 gpurun_out/test_${t}.log; exit 1; }
for d in 0 1 2 3; do
DMLAB_STEM_DIAG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${t}_$d -o run -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof_${t}_$d.log 2>&1 || exit 1
echo "diag $d: $(python tools/prof_summary.py gpurun_out/prof_${t}_$d/run_results.db 8 | grep -i -E 'stem_wgrad|stem_conv')"
done
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 80 --warmup 10 > gpurun_out/b_${t}.json 2>gpurun_out/b_${t}.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/b_${t}.json')); print('$tag', d['value'], d['ms_per_step'])" | tee -a gpurun_out/bench_$t.txt
}
for r in 1 2; do
  run ws1 DMLAB_STEM_WS=1
  run ws0 DMLAB_STEM_WS=0
done
