# Ad-hoc GPU step (overwritten per experiment): layer-1 identity-block dgrads (res64 with the
# fused skip add) reducing the previous block's / the stem's BN sums, on vs off.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3 4; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
DMLAB_NO_RES64_ADD_RED=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_noadd_$tag.json 2>> gpurun_out/bench_noadd_$tag.err || exit 1
done
python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for f in (f"gpurun_out/bench_{t}.json", f"gpurun_out/bench_noadd_{t}.json"):
    v = [json.loads(l)["value"] for l in open(f)]
    print(f, [round(x) for x in v], round(sum(v) / len(v)))
PY
