# Ad-hoc GPU step (overwritten per experiment): layer-1 wgrad on main vs side stream, same box.
set -o pipefail
tag=${1:-tmp}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_$tag.json 2>> gpurun_out/bench_$tag.err || exit 1
DMLAB_WRES64_MAIN=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 >> gpurun_out/bench_main_$tag.json 2>> gpurun_out/bench_main_$tag.err || exit 1
done
cut -c1-160 gpurun_out/bench_$tag.json gpurun_out/bench_main_$tag.json
