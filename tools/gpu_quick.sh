# Targeted GPU check: selected test files, bench, per-kernel profile.
#   gpurun -- bash tools/gpu_quick.sh <tag> "<pytest args>"
set -o pipefail
tag=${1:-q}
tests=${2:-tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$tag.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$tag -o prof -- \
    python bench.py --steps 7 --warmup 3 --graph 0 > gpurun_out/prof_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$tag.log; cat gpurun_out/bench_$tag.json
exit $rc
