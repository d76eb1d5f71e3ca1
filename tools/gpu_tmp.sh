# Ad-hoc GPU step (overwritten per experiment): BN-backward reduction in the data-gradient
# epilogues incl. layer2's cfg 42 halo tile -- kernel + model tests, interleaved A/B.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_native_resnet_kernels.py -k "bn_reduce or masked_add or halo" \
    > gpurun_out/pytest_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_$tag.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_native_resnet_model.py > gpurun_out/pytest_model_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_model_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_model_$tag.log
for i in 1 2 3; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
DMLAB_NO_DGRAD_RED=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_nored_$tag.json 2>> gpurun_out/bench_nored_$tag.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$tag -o tr -- \
    python bench.py --steps 4 --warmup 2 > gpurun_out/trace_$tag.log 2>&1 || exit 1
python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for f in (f"gpurun_out/bench_{t}.json", f"gpurun_out/bench_nored_{t}.json"):
    v = [json.loads(l)["value"] for l in open(f)]
    print(f, [round(x) for x in v], round(sum(v) / len(v)))
PY
