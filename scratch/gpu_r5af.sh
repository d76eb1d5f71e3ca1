set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_conv.py --batch 1024 --iters 10 --cfgs 13,15,42,90,91,92,93 --passes fwd,dgrad --shapes l2_3x3s2,l2_down,l3_3x3s2,l3_down,l4_down > gpurun_out/r5af_conv.jsonl 2> gpurun_out/r5af_conv.err; echo "conv rc=$?"; wc -l gpurun_out/r5af_conv.jsonl; tail -3 gpurun_out/r5af_conv.err
