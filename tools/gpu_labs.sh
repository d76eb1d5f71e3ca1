# GPU step: multi-rank readiness tests, lab-4 pipeline bench (both transports), a HIP API trace
# of the 2-rank xGMI pipeline (host syncs per step), and the GPU lab report (b, c, e).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3c -o prof -- \
    python bench.py --steps 10 --warmup 5 > gpurun_out/prof_r3c.log 2>&1 || exit 1
tail -1 gpurun_out/prof_r3c.log
timeout -k 10 1000 python -u -m pytest tests/test_multiproc_gpu.py -x -v --timeout 280 --timeout-method thread \
    -k "xgmi_many or bf16 or ddp_xgmi_graph or lenet_fused or pipeline_xgmi or bench_lenet" > gpurun_out/pytest_mp2.log 2>&1
rc=$?; tail -16 gpurun_out/pytest_mp2.log; [ $rc -ne 0 ] && exit $rc
for tr in xgmi pg; do
  timeout -k 10 900 python tools/bench_pipeline.py --device cuda --transport $tr --steps 200 \
      --out gpurun_out/bench_pipeline_r3.jsonl >> gpurun_out/bench_pipeline.log 2>&1 || exit 1
done
cat gpurun_out/bench_pipeline_r3.jsonl
P=$(python -c 'import socket; s = socket.socket(); s.bind(("127.0.0.1", 0)); print(s.getsockname()[1])')
export DMLAB_BACKEND=gloo
timeout -k 10 300 rocprofv3 --hip-trace --output-format csv -d gpurun_out/prof_pipe_r0 -o prof -- \
    python -m dmlab.tasks.task4 --mode pipeline --n_devices 2 --rank 0 --master_port $P --device cuda \
    --synthetic --transport xgmi --micro 4 --max-steps 200 --epochs 1 --no-test > gpurun_out/prof_pipe_r0.log 2>&1 &
p0=$!
timeout -k 10 300 rocprofv3 --hip-trace --output-format csv -d gpurun_out/prof_pipe_r1 -o prof -- \
    python -m dmlab.tasks.task4 --mode pipeline --n_devices 2 --rank 1 --master_port $P --device cuda \
    --synthetic --transport xgmi --micro 4 --max-steps 200 --epochs 1 --no-test > gpurun_out/prof_pipe_r1.log 2>&1 &
p1=$!
wait $p0; r0=$?; wait $p1; r1=$?
[ $r0 -ne 0 ] || [ $r1 -ne 0 ] && { tail -5 gpurun_out/prof_pipe_r0.log gpurun_out/prof_pipe_r1.log; exit 1; }
unset DMLAB_BACKEND
python tools/hip_sync_count.py gpurun_out/prof_pipe_r0 gpurun_out/prof_pipe_r1 --steps 200 | tee gpurun_out/pipe_hip_syncs.jsonl
timeout -k 10 1200 python tools/lab_report.py --device cuda --only b,c,e --world-sizes 2 \
    --out gpurun_out/labs_gpu > gpurun_out/lab_report_gpu.log 2>&1 || { tail -30 gpurun_out/lab_report_gpu.log; exit 1; }
tail -3 gpurun_out/lab_report_gpu.log
