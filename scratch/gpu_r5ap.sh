set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5ap_gputests.log 2>&1; rc=$?; echo "gputests rc=$rc"; tail -3 gpurun_out/r5ap_gputests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ap_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r5ap_smoke.log
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/r5ap_bench$i.log 2>/dev/null; echo "bench rc=$? $(tail -1 gpurun_out/r5ap_bench$i.log | cut -c1-200) $(tail -1 gpurun_out/r5ap_bench$i.log | grep -o "param_checksum[^]]*")"; done
timeout -k 10 300 python bench.py --model lenet > gpurun_out/r5ap_lenet.log 2>/dev/null; echo "lenet rc=$? $(tail -1 gpurun_out/r5ap_lenet.log | cut -c1-200)"
