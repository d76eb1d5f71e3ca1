# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=s5l
DMLAB_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 tools/bench_allreduce.py --iters 10 --max-mb 16 > gpurun_out/ar_$t.jsonl 2> gpurun_out/ar_$t.err || { tail -30 gpurun_out/ar_$t.err; exit 1; }
cat gpurun_out/ar_$t.jsonl
