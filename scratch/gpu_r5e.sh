set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r5e_$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -4 gpurun_out/r5e_$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abort after $name"; exit $rc; fi
}
step stem 400 python -u -m pytest tests/test_stem_fused.py -m gpu -v --timeout 200 --timeout-method thread
step benchA 300 python bench.py --steps 20 --warmup 5
DMLAB_STEM_FUSED=1 step benchB 300 python bench.py --steps 20 --warmup 5
export DMLAB_STEM_FUSED=1 AMD_SERIALIZE_KERNEL=3
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5e -o prof -- python bench.py --steps 4 --warmup 2 --phases 0
f=$(find gpurun_out/prof_r5e -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" 6 > gpurun_out/r5e_profsum.txt 2>&1; echo "summary rc=$?"
