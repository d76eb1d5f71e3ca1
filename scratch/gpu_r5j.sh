set -o pipefail
export TMPDIR=/tmp
for ab in 0 5; do
  echo "ablate=$ab"; DMLAB_STEM_TRACE=1 DMLAB_STEM_ABLATE=$ab timeout -k 10 120 python tools/stem_one.py --dtype u8 --iters 1 2>&1 | grep -E "trace|stem B|phase2" | tail -3
done
