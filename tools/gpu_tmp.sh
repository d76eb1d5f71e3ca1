# Scratch GPU session script (overwritten per experiment).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${1:-bytes}
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${t}_f -o pmc -- python bench.py --steps 3 --warmup 2 > gpurun_out/${t}_f.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${t}_w -o pmc -- python bench.py --steps 3 --warmup 2 > gpurun_out/${t}_w.log 2>&1
ls gpurun_out/${t}_f gpurun_out/${t}_w
