set -o pipefail
export TMPDIR=/tmp
for r in 1 2 3; do for g in 256 240 224; do
  echo "grid=$g $(DMLAB_STEM_GRID=$g timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d.get("param_checksum"))')" || exit 1
done; done
