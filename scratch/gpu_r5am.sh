set -o pipefail
export TMPDIR=/tmp
for r in 1 2 3; do for b in 512 384 640 768; do
  echo "blocks=$b $(DMLAB_WGRAD_BLOCKS=$b timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])')" || exit 1
done; done
