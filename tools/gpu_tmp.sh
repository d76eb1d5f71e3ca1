# Ad-hoc GPU step (overwritten per experiment): workgroup cap of the BN-backward apply pass.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
for G in 4096 2048 8192 1024; do
DMLAB_BN_BWD_GRID=$G timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_g${G}_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
done
done
python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for G in (4096, 2048, 8192, 1024):
    v = [json.loads(l)["value"] for l in open(f"gpurun_out/bench_g{G}_{t}.json")]
    print(G, [round(x) for x in v], round(sum(v) / len(v)))
PY
