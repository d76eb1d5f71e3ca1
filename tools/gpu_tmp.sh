# Ad-hoc GPU step (overwritten per experiment): halo-pipe items-per-block sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for ipb in 4 1 0; do
  DMLAB_HPIPE_IPB=$ipb timeout -k 10 300 python -u -m pytest tests/test_native_resnet_kernels.py -x -q --timeout 120 --timeout-method thread -k hpipe > gpurun_out/pytest_hpipe_$ipb.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_hpipe_$ipb.log; [ $rc -ne 0 ] && exit $rc
done
out=gpurun_out/bench_conv_hpipe_ipb.jsonl; : > $out
for ipb in 0 1 2 4 8; do
  echo "IPB=$ipb" >> $out
  DMLAB_HPIPE_IPB=$ipb timeout -k 10 300 python tools/bench_conv.py --batch 1024 --shapes l1_3x3,l2_3x3 \
      --cfgs 39,42,94,95 --passes fwd,dgrad --iters 20 >> $out 2>> gpurun_out/bench_conv.err || exit 1
done
cat $out
out=gpurun_out/bench_ab_hpipe2.jsonl; : > $out
for v in "DMLAB_NO_HPIPE=1" "DMLAB_HPIPE_IPB=2" "DMLAB_HPIPE_IPB=4" "DMLAB_HPIPE_IPB=8" "DMLAB_NO_HPIPE=1" "DMLAB_HPIPE_IPB=4"; do
  echo "$v" >> $out
  env $v timeout -k 10 300 python bench.py --steps 30 --warmup 10 >> $out 2>> gpurun_out/bench_ab.err || exit 1
done
python - <<'PY'
import json
for l in open('gpurun_out/bench_ab_hpipe2.jsonl'):
    l = l.strip()
    if l.startswith('{'):
        r = json.loads(l); print(r['value'], r['ms_per_step'])
    else: print(l, end=' ')
PY
