set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_conv.py --batch 1024 --iters 10 --cfgs 15,42,80,90 --wcfgs v2,h9,h3,q8 > gpurun_out/r5ae_conv.jsonl 2> gpurun_out/r5ae_conv.err; echo "conv rc=$?"; wc -l gpurun_out/r5ae_conv.jsonl
