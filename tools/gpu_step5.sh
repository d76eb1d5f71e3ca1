set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest5.log 2>&1
rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench5.json 2> gpurun_out/bench5.err
exit $rc
