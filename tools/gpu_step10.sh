set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_graph_capture.py -q -x > gpurun_out/pytest10.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench10.json 2> gpurun_out/bench10.err
timeout -k 10 300 python bench.py --model lenet --steps 500 --warmup 20 > gpurun_out/bench10_lenet.json 2> gpurun_out/bench10_lenet.err
timeout -k 10 300 python bench.py --model lenet --steps 500 --warmup 20 --graph 0 > gpurun_out/bench10_lenet_eager.json 2>&1
