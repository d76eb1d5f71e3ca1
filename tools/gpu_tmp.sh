# Ad-hoc GPU step (overwritten per experiment): BN pass loads-in-flight A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DMLAB_BNR_U=8 DMLAB_BNA_U=8 DMLAB_BNF_U=8 timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py tests/test_native_resnet_model.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bn or model or resnet" > gpurun_out/pytest_bnu.log 2>&1 || { tail -20 gpurun_out/pytest_bnu.log; exit 1; }
tail -1 gpurun_out/pytest_bnu.log
out=gpurun_out/bnu_ab.jsonl; : > $out
for cfg in "4 4 4" "8 4 4" "4 8 4" "4 4 8" "8 8 8" "4 4 4" "8 8 8"; do
  set -- $cfg
  echo "reduceU=$1 applyU=$2 fwdU=$3" >> $out
  DMLAB_BNR_U=$1 DMLAB_BNA_U=$2 DMLAB_BNF_U=$3 timeout -k 10 200 python bench.py --steps 40 --warmup 8 >> $out 2>> gpurun_out/bnu_ab.err || exit 1
done
cut -c1-120 $out
