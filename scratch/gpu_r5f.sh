set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r5f_$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/r5f_$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abort after $name"; exit $rc; fi
}
step stem 400 python -u -m pytest tests/test_stem_fused.py -m gpu -v --timeout 200 --timeout-method thread
step one_f32 120 python tools/stem_one.py --dtype f32
step one_u8 120 python tools/stem_one.py --dtype u8
for p in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  n=$(echo $p | cut -c1-12 | tr ' ' _)
  step pmc_$n 90 rocprofv3 --pmc $p --output-format csv -d gpurun_out/pmc_r5f_$n -o pmc -- python tools/stem_one.py --dtype f32 --iters 2
done
