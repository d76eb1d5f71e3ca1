set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for ab in 0 3 7 15; do
  DMLAB_STEM_ABLATE=$ab timeout -k 10 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_r5h_$ab -o pmc -- python tools/stem_one.py --dtype u8 --iters 2 > gpurun_out/r5h_$ab.log 2>&1 || exit 1
done
echo done
