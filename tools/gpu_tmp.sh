# Ad-hoc GPU step (overwritten per experiment): side-stream knobs re-checked with the pipe convs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/bench_ab_defer_r3.jsonl; : > $out
for v in "X=0" "DMLAB_DEFER_WGRAD=1" "DMLAB_DEFER_WGRAD=2" "DMLAB_DEFER_WGRAD=4" \
         "X=0" "DMLAB_DEFER_WGRAD=1" "DMLAB_DEFER_WGRAD=2" "DMLAB_DEFER_WGRAD=4"; do
  echo "$v" >> $out
  env $v timeout -k 10 300 python bench.py --steps 30 --warmup 10 >> $out 2>> gpurun_out/bench_ab.err || exit 1
done
python - <<'PY'
import json
for l in open('gpurun_out/bench_ab_defer_r3.jsonl'):
    l = l.strip()
    if l.startswith('{'):
        r = json.loads(l); print(r['value'], r['ms_per_step'])
    else: print(l, end=' ')
PY
