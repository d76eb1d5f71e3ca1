set -o pipefail
export TMPDIR=/tmp
run() { echo "$1 $(env $1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d.get("final_loss"))')"; }
for r in 1 2; do
  run DMLAB_WRES64_8=5 && run DMLAB_WRES64_8=4 && run DMLAB_WRES64_8=6 && run DMLAB_WRES64_TAIL8=6 && run DMLAB_WRES64_8=3 || exit 1
done
