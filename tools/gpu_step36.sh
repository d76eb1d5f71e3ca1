set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_multiproc_gpu.py -m gpu -q -x > gpurun_out/pytest36.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench36_g.json 2> gpurun_out/bench36_g.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench36_e.json 2> gpurun_out/bench36_e.err
