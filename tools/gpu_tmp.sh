# Ad-hoc GPU step (overwritten per experiment): host enqueue time of the ResNet step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/host_lead.py --steps 30 --warmup 5 --profile gpurun_out/host2.prof > gpurun_out/host_lead.json 2>&1 && \
python -c "
import pstats
p = pstats.Stats('gpurun_out/host2.prof')
p.sort_stats('tottime').print_stats(45)
p.sort_stats('cumtime').print_stats(45)
" > gpurun_out/host_prof2.txt 2>&1
rc=$?
cat gpurun_out/host_lead.json
exit $rc
