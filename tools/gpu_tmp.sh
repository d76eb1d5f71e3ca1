# Ad-hoc GPU step (overwritten per experiment): halo-pipe on layer 2 only, persistent vs runs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/bench_ab_hpipe3.jsonl; : > $out
for v in "DMLAB_NO_HPIPE=1" "DMLAB_HPIPE_IPB=0" "DMLAB_HPIPE_IPB=1" "DMLAB_NO_HPIPE=1" "DMLAB_HPIPE_IPB=0" "DMLAB_HPIPE_IPB=1"; do
  echo "$v" >> $out
  env $v timeout -k 10 300 python bench.py --steps 30 --warmup 10 >> $out 2>> gpurun_out/bench_ab.err || exit 1
done
python - <<'PY'
import json
for l in open('gpurun_out/bench_ab_hpipe3.jsonl'):
    l = l.strip()
    if l.startswith('{'):
        r = json.loads(l); print(r['value'], r['ms_per_step'])
    else: print(l, end=' ')
PY
