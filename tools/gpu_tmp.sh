# Ad-hoc GPU step (overwritten per experiment): repeatability of the fused-skip step.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3 4; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
done
DMLAB_NO_FUSED_SKIP=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_nofs_$tag.json 2>> gpurun_out/bench_nofs_$tag.err || exit 1
python - <<'PY'
import json,sys
for f in ("gpurun_out/bench_fs3.json","gpurun_out/bench_nofs_fs3.json"):
    for l in open(f):
        d=json.loads(l); print(f, d["value"], d["ms_per_step"], d.get("peak_mem_gb"))
PY
