# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${1:-tail}
timeout -k 10 600 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$t.log 2>&1 || { tail -40 gpurun_out/pytest_$t.log; exit 1; }
tail -2 gpurun_out/pytest_$t.log
timeout -k 10 300 python tools/bench_conv.py --batch 512 --iters 20 --cfgs 41 --passes fwd,dgrad --shapes l3_3x3,l4_3x3 > gpurun_out/conv_${t}_on.jsonl 2>&1 && DMLAB_TAIL_SPLIT=0 timeout -k 10 300 python tools/bench_conv.py --batch 512 --iters 20 --cfgs 41 --passes fwd,dgrad --shapes l3_3x3,l4_3x3 > gpurun_out/conv_${t}_off.jsonl 2>&1 && cat gpurun_out/conv_${t}_on.jsonl gpurun_out/conv_${t}_off.jsonl
for f in 1 0 1 0 1 0; do
DMLAB_TAIL_SPLIT=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${t}_$f.json 2> gpurun_out/bench_${t}_$f.err || { tail -20 gpurun_out/bench_${t}_$f.err; exit 1; }
echo "tail_split $f: $(python -c "import json;d=json.load(open('gpurun_out/bench_${t}_$f.json'));print(d['value'], d['ms_per_step'], d['final_loss'])")"
done
for v in "split igemm 4" "fused dy 4" "split igemm 8"; do
set -- $v
DMLAB_STEM_BWD=$1 DMLAB_STEM_WGRAD=$2 DMLAB_STEM_SPLIT=$3 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$t.json 2> gpurun_out/bench_$t.err || { tail -20 gpurun_out/bench_$t.err; exit 1; }
echo "$v: $(python -c "import json;d=json.load(open('gpurun_out/bench_$t.json'));print(d['value'], d['ms_per_step'], d['final_loss'])")"
done
