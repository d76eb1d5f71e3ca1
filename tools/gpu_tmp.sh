set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -m gpu -x -q -k "42 or 43" --timeout 120 --timeout-method thread > gpurun_out/pytest_q5.log 2>&1 && \
timeout -k 10 300 python tools/bench_conv.py --cfgs 20,42,38,43 --passes fwd,dgrad --shapes l2_3x3,l3_3x3,l4_3x3 > gpurun_out/bconv_q5.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_q5.log; grep shape gpurun_out/bconv_q5.log; exit $rc
