set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r5ab_$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/r5ab_$name.log
  if [ $rc -ne 0 ]; then echo "abort after $name"; exit $rc; fi
}
step ktrace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r5ab -o k -- python bench.py --steps 6 --warmup 3 --phases 0
f=$(find gpurun_out/prof_r5ab -name "*kernel_trace.csv" | head -1); python tools/step_trace.py "$f" > gpurun_out/r5ab_step.txt 2>&1; echo "steptrace rc=$?"
export AMD_SERIALIZE_KERNEL=3
step profbench 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5ab_ser -o prof -- python bench.py --steps 4 --warmup 2 --phases 0
unset AMD_SERIALIZE_KERNEL
f=$(find gpurun_out/prof_r5ab_ser -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py "$f" 6 > gpurun_out/r5ab_profsum.txt 2>&1; echo "sum rc=$?"
