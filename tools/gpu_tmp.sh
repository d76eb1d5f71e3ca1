# Ad-hoc GPU step (overwritten per experiment): layers 2-4 weight-gradient block budget
# (DMLAB_WGRAD_BLOCKS) now that layer 1's wgrad leaves CUs to the main stream.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
for B in 512 384 256; do
DMLAB_WGRAD_BLOCKS=$B timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_b${B}_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
done
done
python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for B in (512, 384, 256):
    v = [json.loads(l)["value"] for l in open(f"gpurun_out/bench_b{B}_{t}.json")]
    print(B, [round(x) for x in v], round(sum(v) / len(v)))
PY
