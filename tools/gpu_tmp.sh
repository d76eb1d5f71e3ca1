# Ad-hoc GPU step (overwritten per experiment): pipelined conv tiles (cfg 90-92) vs the halo/v3 tiles.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -k "pipe" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_pipe.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_conv.py --batch 256 --passes fwd,dgrad --cfgs 15,41,43,90,91,92 \
   --shapes l2_3x3,l3_3x3,l4_3x3,l3_3x3s2,l4_3x3s2,l3_down,gemm_k2048_n256 > gpurun_out/bench_pipe.jsonl 2>&1 && \
timeout -k 10 200 python tools/gemm_ceiling.py > gpurun_out/gemm_ceiling.jsonl 2>&1
rc=$?
cat gpurun_out/bench_pipe.jsonl; grep -E "l3_3x3\"|gemm_k2048" gpurun_out/gemm_ceiling.jsonl
exit $rc
