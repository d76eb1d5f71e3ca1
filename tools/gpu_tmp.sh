# Ad-hoc GPU step (overwritten per experiment): stem pool kernel timing.
set -o pipefail
mkdir -p gpurun_out
for g in 1 0 1 0; do DMLAB_POOL_GENERIC=$g timeout -k 10 120 python tools/time_pool.py 2>&1 | grep -v amdgpu.ids | sed "s/^/generic=$g /" >> gpurun_out/time_pool.txt || exit 1; done
cat gpurun_out/time_pool.txt
