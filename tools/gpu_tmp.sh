# Ad-hoc GPU step (overwritten per experiment): the step's last layer-1 weight gradient on all
# CUs (it overlaps the stem's backward, not a dgrad chain) vs 5/8 like the others.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3 4; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
DMLAB_TAIL_WGRAD_FULL=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_off_$tag.json 2>> gpurun_out/bench_off_$tag.err || exit 1
done
python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for f in (f"gpurun_out/bench_{t}.json", f"gpurun_out/bench_off_{t}.json"):
    v = [json.loads(l)["value"] for l in open(f)]
    print(f, [round(x) for x in v], round(sum(v) / len(v)))
PY
