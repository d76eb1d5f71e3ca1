# Ad-hoc GPU step (overwritten per experiment): HIP API trace of the ResNet step (host timing).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/prof_api -o prof -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof_api.log 2>&1
rc=$?
ls gpurun_out/prof_api
exit $rc
