# Ad-hoc GPU step (overwritten per experiment): host run-ahead bound (Program.max_inflight)
# vs throughput and reserved device memory.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
for K in 2 1 4 0; do
DMLAB_MAX_INFLIGHT=$K timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_k${K}_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
done
done
python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for K in (2, 1, 4, 0):
    for l in open(f"gpurun_out/bench_k{K}_{t}.json"):
        d = json.loads(l)
        print(K, d["value"], d["peak_mem_gb"], d["peak_alloc_gb"], d["alloc_retries"])
PY
