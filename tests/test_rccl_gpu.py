"""The RCCL (ProcessGroupNCCL) data-parallel path, run for real on the one-GPU box.

Two ranks cannot share a GPU under RCCL, but a 1-RANK communicator is legal, and with
``DDP(force_comm=True)`` the world-size-1 run takes the whole multi-rank path: native C++
reducer, bucket hooks on the weight-gradient side stream, ``pg->allreduce`` per bucket,
bf16 communication buffers, buffer broadcasts, RCCL inside a captured hipGraph.  Each
scenario runs in its own process (tests/rccl_one_rank_worker.py), so a communicator never
outlives its test.  Reference DP call pattern: codes/task3/dist_utils.py:40-46.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

from dist_helpers import free_port

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _run(scenario, timeout=240):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "-u", str(ROOT / "tests" / "rccl_one_rank_worker.py"),
                        scenario], env=env, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    res = json.loads(lines[-1])
    assert res.get("ok"), res
    return res


def test_rccl_resnet_ddp_fp32_bitwise():
    res = _run("resnet_fp32")
    assert res["launched"] == res["expect_launched"] and res["buckets"] >= 2


def test_rccl_resnet_ddp_bf16_comm():
    res = _run("resnet_bf16")
    assert res["launched"] > 0


def test_rccl_lenet_fused_step_in_hipgraph():
    res = _run("lenet_graph")
    assert res["eager_launched"] > 0


def test_rccl_broadcast_buffers_and_init():
    _run("buffers")


def test_rccl_p2p_self_is_unsupported():
    _run("p2p_self")


def test_rccl_grad_aggregator():
    _run("aggregator")


def _bench(args, timeout=400):
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "bench.py"),
           "--gpus", "1", "--force-comm", "1"] + args
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_force_comm_resnet():
    """bench.py under torchrun at one rank with the RCCL path forced: every bucket
    all-reduced, the self-check fields present and consistent."""
    res = _bench(["--steps", "3", "--warmup", "1", "--res", "64", "--batch", "16",
                  "--phases", "2"])
    assert res["rccl_world"] == 1 and res["distinct_gpus"] == 1
    assert res["replicas_in_sync"] is True and res["buckets_launched"] > 0
    assert res["config"]["process_group"] == "nccl" and "forced" in res["config"]["ddp"]
    assert set(res["phases_ms"]) == {"fwd", "bwd_compute", "comm_exposed", "opt"}
    assert res["config"]["sampler"] == "MySampler(partition)"


def test_bench_force_comm_lenet_graph():
    """The fused LeNet step with the RCCL all-reduce captured in a hipGraph (what bench does
    at ws > 1 on RCCL), batches drawn on the device through the sampler's epoch order."""
    res = _bench(["--model", "lenet", "--steps", "50", "--warmup", "5"])
    assert res["config"]["hip_graph"] is True and res["config"]["fused_step"] is True
    assert res["config"]["hip_graph_steps"] == 25  # 25 steps (25 all-reduces) per replay
    assert res["replicas_in_sync"] is True and res["value"] > 0


def _task2(nproc, args, extra_env=None, timeout=300):
    import re

    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="2", **(extra_env or {}))
    cmd = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
            str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(free_port())]
           if nproc > 1 else [sys.executable])
    if nproc == 1:
        args = args + ["--master_port", str(free_port())]
    r = subprocess.run(cmd + ["-m", "dmlab.tasks.task2", "--device", "cuda", "--synthetic",
                              "--epochs", "1", "--max-steps", "60", "--no-test"] + args,
                       env=env, capture_output=True, text=True, timeout=timeout, cwd=str(ROOT))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    losses = [float(v) for v in re.findall(r"Device: 0 epoch: \d+, iters:\s+\d+, loss: (\d+\.\d+)",
                                           r.stdout)]
    comm = float(re.search(r"Total communication time: ([\d.eE+-]+)", r.stdout).group(1))
    return losses, comm


def test_task2_rccl_one_rank_forced():
    """Lab 2's aggregation through a 1-rank RCCL communicator (task2 --backend nccl
    --force-comm): every collective issued and timed on the device path."""
    for agg in ("allreduce", "allgather"):
        losses, comm = _task2(1, ["--backend", "nccl", "--force-comm", "--aggregation", agg])
        assert len(losses) == 3 and comm > 0


def test_task2_xgmi_kernel_two_ranks():
    """Lab 2's all-reduce on the one-shot xGMI peer-memory kernel, two ranks sharing the GPU."""
    losses, comm = _task2(2, ["--aggregation", "allreduce_xgmi"], {"DMLAB_BACKEND": "gloo"})
    assert len(losses) == 3 and losses[-1] < losses[0] + 0.5 and comm > 0
