# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${1:-fin}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$t.log 2>&1 || { tail -40 gpurun_out/pytest_$t.log; exit 1; }
tail -2 gpurun_out/pytest_$t.log
for f in 1 0 1 0 1 0; do
DMLAB_FUSED_FIN=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${t}_$f.json 2> gpurun_out/bench_${t}_$f.err || { tail -20 gpurun_out/bench_${t}_$f.err; exit 1; }
echo "fused_fin $f: $(python -c "import json;d=json.load(open('gpurun_out/bench_${t}_$f.json'));print(d['value'], d['ms_per_step'], d['final_loss'])")"
done
for b in 768 1024; do
timeout -k 10 300 python bench.py --steps 15 --warmup 5 --batch $b > gpurun_out/bench_${t}_b$b.json 2> gpurun_out/bench_${t}_b$b.err || { tail -20 gpurun_out/bench_${t}_b$b.err; exit 1; }
echo "batch $b: $(python -c "import json;d=json.load(open('gpurun_out/bench_${t}_b$b.json'));print(d['value'], d['ms_per_step'])")"
done
