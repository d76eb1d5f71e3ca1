"""Two ranks sharing the box's single GPU (gloo group; device tensors staged
through the host where gloo needs it): the DDP reducer and the P2P pipeline
driving the NATIVE HIP kernels, checked against a single-process run."""
import os

import pytest
import torch
import torch.nn.functional as F

from dist_helpers import free_port

pytestmark = pytest.mark.gpu


def _entry(rank, ws, port, kind, q):
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK="0")
    import torch.distributed as dist

    from dmlab.models import Net, SubNetConv, SubNetFC
    from dmlab.nn import cross_entropy, CrossEntropyLoss
    from dmlab.optim import SGD

    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        g = torch.Generator().manual_seed(5)
        X = torch.rand(16, 1, 28, 28, generator=g).to(dev)
        Y = torch.randint(0, 10, (16,), generator=g).to(dev)
        torch.manual_seed(0)
        ref = Net().to(dev)
        ropt = SGD(ref.parameters(), lr=0.1, momentum=0.9)
        if kind == "xgmi":
            from dmlab.parallel.xgmi import XGMIAllReduce

            ar = XGMIAllReduce(cap=(1 << 20) + 8)
            err = 0.0
            # one-shot and two-shot interleaved on one instance (shared epochs and parity
            # halves); two-shot sizes cover the float4 path (n % 4 == 0, aligned), the
            # scalar path (odd n, misaligned view) and slices shorter than the grid
            cases = [(1, "one_shot"), (1000, "two_shot"), (51902, "one_shot"),
                     (65536, "two_shot"), (7, "two_shot"), ((1 << 20) + 8, "two_shot"),
                     (300001, "two_shot"), (3, "one_shot"), (524288, "two_shot"),
                     (1 << 19, None), (4096, None)]  # instance default: auto
            for it, (n, algo) in enumerate(cases):
                t = torch.arange(n, device=dev, dtype=torch.float32) * (rank + 1) + it
                exp = torch.arange(n, device=dev, dtype=torch.float32) * (ws * (ws + 1) // 2) \
                    + ws * it
                if it == 6:  # a view 4 B into its storage: not 16-B aligned
                    t = torch.cat([torch.zeros(1, device=dev), t])[1:]
                if it % 2:
                    out = ar(t.clone(), scale=0.5, algo=algo)  # scaled copy
                else:
                    out = ar(t, algo=algo)  # in place
                ref_v = exp * (0.5 if it % 2 else 1.0)
                err = max(err, ((out - ref_v).abs().max() / ref_v.abs().max().clamp_min(1)).item())
            ar.check()
            ar.close()
        elif kind == "xgmi_graph":
            # the all-reduce captured into a hipGraph and replayed: the epoch (flag value and
            # parity half) lives on the device, so every replay is a fresh, correct call
            from dmlab.parallel.xgmi import XGMIAllReduce

            ar = XGMIAllReduce(cap=4096)
            n = 4000
            src = torch.zeros(n, device=dev)
            dst = torch.zeros(n, device=dev)
            ar(src, out=dst)  # eager call before capture (epoch 1)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                ar(src, out=dst, scale=0.5)
            err = 0.0
            base = torch.arange(n, device=dev, dtype=torch.float32)
            for it in range(6):
                src.copy_(base * (rank + 1) + it)
                graph.replay()
                want = 0.5 * (base * (ws * (ws + 1) // 2) + ws * it)
                err = max(err, ((dst - want).abs().max() / want.abs().max()).item())
            assert ar.epoch == 7, ar.epoch  # 1 eager + 6 replays (capture does not run it)
            ar.check()
            ar.poll()
            ar.close()
        elif kind in ("ddp_resnet", "ddp_resnet_xgmi2", "ddp_resnet_bf16"):
            # ResNet-18 (bf16 native kernels, conv weight gradients on the side stream):
            # the DDP-averaged gradient == the mean of the two per-shard gradients computed
            # one after the other in this process (BN statistics are per shard either way)
            from dmlab.models import ResNet18
            from dmlab.parallel import DDP

            gr = torch.Generator().manual_seed(7)
            Xr = torch.rand(8, 3, 32, 32, generator=gr).to(dev)
            Yr = torch.randint(0, 10, (8,), generator=gr).to(dev)
            torch.manual_seed(0)
            model = ResNet18(num_classes=10).to(dev)
            if kind == "ddp_resnet":
                ddp = DDP(model)
            elif kind == "ddp_resnet_bf16":
                # bf16 gradient communication from the side-stream (stream_ok) bucket hooks:
                # the persistent bf16 comm buffer is written on the weight-gradient stream
                ddp = DDP(model, comm_dtype=torch.bfloat16, side_stream_hooks=True)
                assert ddp.side_stream_hooks
            else:  # every bucket (4 MB first, then 25 MB) through the two-shot xGMI kernel
                ddp = DDP(model, small_allreduce="xgmi", small_cap_mb=1e4, xgmi_algo="two_shot")
                assert ddp._xgmi is not None and ddp._xgmi.cap >= max(
                    b.hi - b.lo for b in ddp.buckets)
            mopt = SGD(model.parameters(), lr=0.1)
            mopt.zero_grad()
            cross_entropy(ddp(Xr[rank * 4:(rank + 1) * 4]), Yr[rank * 4:(rank + 1) * 4]).backward()
            g_ddp = model.flat.grad.clone()
            torch.manual_seed(0)
            rmodel = ResNet18(num_classes=10).to(dev)
            rsgd = SGD(rmodel.parameters(), lr=0.1)
            gs = []
            for k in range(2):
                rsgd.zero_grad()
                cross_entropy(rmodel(Xr[k * 4:(k + 1) * 4]), Yr[k * 4:(k + 1) * 4]).backward()
                gs.append(rmodel.flat.grad.clone())
            want = (gs[0] + gs[1]) / 2
            err = ((g_ddp - want).abs().max() / want.abs().max().clamp_min(1e-12)).item()
            if kind == "ddp_resnet_bf16":  # bf16 rounding of each rank's gradient: ~2^-8
                rel = ((g_ddp - want).norm() / want.norm()).item()
                assert rel < 8e-3, rel
                err = 0.0 if err < 2e-2 else err
        elif kind in ("ddp", "ddp_xgmi"):
            from dmlab.parallel import DDP

            torch.manual_seed(0)
            model = Net().to(dev)
            ddp = DDP(model, small_allreduce="xgmi" if kind == "ddp_xgmi" else None)
            assert (ddp._xgmi is not None) == (kind == "ddp_xgmi")
            opt = SGD(model.parameters(), lr=0.1, momentum=0.9)
            ddp.fold_average_into(opt)
            for _ in range(2):
                opt.zero_grad()
                cross_entropy(ddp(X[rank * 8:(rank + 1) * 8]), Y[rank * 8:(rank + 1) * 8]).backward()
                opt.step()
                ropt.zero_grad()
                cross_entropy(ref(X), Y).backward()
                ropt.step()
            err = max((a - b).abs().max().item() for a, b in zip(model.parameters(), ref.parameters()))
        elif kind in ("lenet_fused_ddp", "lenet_fused_ddp_xgmi"):
            # the fused 2-dispatch LeNet step with DDP (grads -> bucket all-reduce -> fused
            # SGD) equals one process on the whole batch
            from dmlab.models.lenet_fused import FusedLeNetStep
            from dmlab.parallel import DDP

            torch.manual_seed(0)
            model = Net().to(dev)
            ddp = DDP(model, small_allreduce="xgmi" if kind.endswith("xgmi") else None)
            opt = ddp.fold_average_into(SGD(model.parameters(), lr=0.1, momentum=0.9))
            step = FusedLeNetStep(model, opt, ddp=ddp)
            for _ in range(3):
                step(X[rank * 8:(rank + 1) * 8], Y[rank * 8:(rank + 1) * 8])
                ropt.zero_grad()
                cross_entropy(ref(X), Y).backward()
                ropt.step()
            err = max((a - b).abs().max().item() for a, b in zip(model.parameters(), ref.parameters()))
        elif kind == "ddp_xgmi_graph":
            # the whole DDP step (Program backward, bucket hooks, xGMI all-reduce kernel, fused
            # SGD) captured into a hipGraph at world size 2 == the same step run eagerly,
            # bit for bit
            from dmlab.parallel import DDP
            from dmlab.utils.graph import CapturedStep

            runs = []
            for captured in (False, True):
                torch.manual_seed(0)
                model = Net().to(dev)
                ddp = DDP(model, small_allreduce="xgmi")
                opt = ddp.fold_average_into(SGD(model.parameters(), lr=0.1, momentum=0.9))
                xs, ys = X[rank * 8:(rank + 1) * 8].clone(), Y[rank * 8:(rank + 1) * 8].clone()

                def train_step(x, y):
                    loss = cross_entropy(ddp(x), y)
                    opt.zero_grad()
                    loss.backward()
                    opt.step()
                    return loss.detach()

                if captured:
                    cap = CapturedStep(train_step, [xs, ys], warmup=2, bind_inputs=True)
                    for _ in range(3):
                        cap(xs, ys)
                else:
                    for _ in range(5):  # the capture warm-up runs 2 eager steps
                        train_step(xs, ys)
                torch.cuda.synchronize()
                ddp.check()
                runs.append([p.detach().clone() for p in model.parameters()])
            err = max((a - b).abs().max().item() for a, b in zip(*runs))
            assert err == 0.0, err
        elif kind in ("pipeline_xgmi", "pipeline_xgmi_gpipe", "pipeline_xgmi_cupart",
                      "pipeline_xgmi_graph"):
            # the native xGMI stage transport (IPC ring, device flags; the two ranks share
            # the GPU here), prefetched receives, 1F1B / GPipe; ``cupart``: every stage on its
            # own half of the CUs (a CU-masked stream), as task4 --cu-partition
            import contextlib

            from dmlab.parallel.pipeline import PipelineStage
            from dmlab.utils.streams import partition_stream

            scope = (torch.cuda.stream(partition_stream(rank, 2, dev)) if kind.endswith("cupart")
                     else contextlib.nullcontext())
            scope.__enter__()
            mod = (SubNetConv() if rank == 0 else SubNetFC()).to(dev)
            sd = {k: v for k, v in ref.state_dict().items()
                  if k.startswith("conv" if rank == 0 else "fc")}
            mod.load_state_dict(sd)
            st = PipelineStage(mod, SGD(mod.parameters(), lr=0.1, momentum=0.9), CrossEntropyLoss(),
                               device=dev, transport="xgmi", timing=True,
                               schedule="gpipe" if kind.endswith("gpipe") else "1f1b")
            xs, ys = (X, Y) if rank == 0 else (None, None)
            for i in range(3):
                if kind.endswith("graph"):  # step 0 eager + capture, then two replays
                    if i == 0:
                        st.capture(xs, ys, n_micro=4, warmup=1)
                    else:
                        st.replay(xs, ys)
                else:
                    st.train_step(xs, ys, n_micro=4)
                ropt.zero_grad()
                cross_entropy(ref(X), Y).backward()
                ropt.step()
            step_ms, comp_ms, bubble = st.step_stats()
            if kind.endswith("graph"):
                assert step_ms > 0.0 and comp_ms is None
            else:
                assert 0.0 <= bubble < 1.0 and comp_ms > 0.0
            st.p2p.check()
            err = max((p - ref.get_parameter(n)).abs().max().item()
                      for n, p in mod.named_parameters())
            st.p2p.close()
            scope.__exit__(None, None, None)
        else:
            from dmlab.parallel.pipeline import PipelineStage

            mod = (SubNetConv() if rank == 0 else SubNetFC()).to(dev)
            sd = {k: v for k, v in ref.state_dict().items()
                  if k.startswith("conv" if rank == 0 else "fc")}
            mod.load_state_dict(sd)
            st = PipelineStage(mod, SGD(mod.parameters(), lr=0.1, momentum=0.9), CrossEntropyLoss(),
                               device=dev)
            for _ in range(2):
                st.train_step(X if rank == 0 else None, Y if rank == 0 else None, n_micro=4)
                ropt.zero_grad()
                cross_entropy(ref(X), Y).backward()
                ropt.step()
            err = max((p - ref.get_parameter(n)).abs().max().item()
                      for n, p in mod.named_parameters())
        q.put((rank, err, None))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("kind", ["ddp", "ddp_xgmi", "ddp_resnet", "ddp_resnet_xgmi2",
                                  "ddp_resnet_bf16", "pipeline",
                                  "xgmi", "xgmi_graph", "lenet_fused_ddp", "lenet_fused_ddp_xgmi",
                                  "ddp_xgmi_graph", "pipeline_xgmi", "pipeline_xgmi_gpipe",
                                  "pipeline_xgmi_cupart", "pipeline_xgmi_graph"])
def test_two_ranks_one_gpu(kind):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    ps = [ctx.Process(target=_entry, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(240)
    res = [q.get() for _ in range(2) if not q.empty()]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert len(res) == 2, res
    for rank, err, tb in res:
        assert tb is None, tb
        assert err < 2e-4, (rank, err)


def test_partition_stream_mask_and_compute():
    """A CU-masked stream reports the mask it was built with and computes correctly; the two
    halves are disjoint and cover every CU."""
    import torch

    from dmlab.ops._native import lib
    from dmlab.utils.streams import partition_stream

    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    masks = []
    for part in range(2):
        st = partition_stream(part, 2)
        m = lib().cu_mask_of(st.cuda_stream, words)
        masks.append(sum(int(w) << (32 * i) for i, w in enumerate(m)))
        a = torch.randn(512, 512, device="cuda")
        with torch.cuda.stream(st):
            c = a @ a
        st.synchronize()
        assert torch.allclose(c, (a.double() @ a.double()).float(), rtol=1e-3, atol=1e-2)
    assert masks[0] & masks[1] == 0
    assert bin(masks[0] | masks[1]).count("1") == ncu


def test_rpc_stages_on_gpu(tmp_path):
    """BASELINE config 4: the reference RPC/RRef programming model with both stage owners
    on the GPU (native HIP kernels inside each stage; the box has one GPU, so both share it)."""
    import re
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    env = dict(os.environ, PYTHONPATH=str(root), OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "3",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m",
                        "dmlab.tasks.task4", "--mode", "rpc", "--device", "cuda", "--synthetic",
                        "--train-samples", "3200", "--epochs", "1", "--lr", "0.05"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout + r.stderr
    ls = [float(x) for x in re.findall(r"loss: (\d+\.\d+)", r.stdout)]
    assert len(ls) == 5 and ls[-1] < ls[0]
    assert "Test set: Accuracy" in r.stdout


def test_bench_two_ranks(tmp_path):
    """bench.py's multi-rank path (env init, barrier-bracketed timing, MAX over ranks, one
    JSON line from rank 0) with two ranks sharing the box's GPU over gloo."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DMLAB_BACKEND="gloo",
                   OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen(
            [sys.executable, str(root / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
             "--res", "64", "--batch", "8"], cwd=tmp_path, env=env, stdout=subprocess.PIPE,
            stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and not [ln for ln in outs[1][0].splitlines() if ln.startswith("{")]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 3 and res["value"] > 0
    assert res["config"]["parallelism"] == "dp2" and res["config"]["global_batch"] == 16
    # the multi-rank self-check (both ranks on this box's one GPU, gloo group)
    assert res["distinct_gpus"] == 1 and res["rccl_world"] is None
    assert res["replicas_in_sync"] is True and res["buckets_launched"] > 0
    assert set(res["phases_ms"]) == {"fwd", "bwd_compute", "comm_exposed", "opt"}
    assert res["config"]["sampler"] == "MySampler(partition)"
    # startup device-path self-checks: the closed-form all-reduce ran; ResNet stays on the
    # process group's all-reduce (no xGMI probe)
    assert res["allreduce_selfcheck"] == "pass"
    assert res["xgmi_selfcheck"] == "skipped" and res["small_allreduce_used"] == "rccl"


@pytest.mark.parametrize("ws", [4, 8])
def test_xgmi_many_ranks_one_gpu(ws):
    """Four and eight ranks (the 8-GPU node's world size, all on this box's one GPU): 'auto'
    picks the two-shot kernel (W >= 3, >= 1 MB) -- W rank slices, reduce-scatter then
    all-gather through W IPC-mapped buffers; every wait in the kernels is bounded, so a
    rank that never arrives sets the timeout flag instead of hanging the GPU.  The ranks find
    that they share one device and shrink their spinning grids by W (8 x 256 two-shot blocks
    do not all fit beside each other: resident blocks would wait on peers that cannot start)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    ps = [ctx.Process(target=_entry, args=(r, ws, port, "xgmi", q)) for r in range(ws)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(240)
    res = [q.get() for _ in range(ws) if not q.empty()]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert len(res) == ws, res
    for rank, err, tb in res:
        assert tb is None, tb
        assert err < 2e-4, (rank, err)


@pytest.mark.parametrize("corrupt", [None, "xgmi:1"])
def test_bench_lenet_two_ranks_graph(tmp_path, corrupt):
    """bench.py --model lenet at 2 ranks (gloo process group on the shared GPU): with the
    xGMI all-reduce kernel the whole DDP step (fused LeNet step, all-reduce, SGD) is captured
    into a hipGraph at world size > 1 (hip_graph: true in the JSON line)."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DMLAB_BACKEND="gloo",
                   OMP_NUM_THREADS="2")
        if corrupt:  # a forced wrong xGMI sum on rank 1: both ranks must fall back together
            env["DMLAB_SELFCHECK_CORRUPT"] = corrupt
        procs.append(subprocess.Popen(
            [sys.executable, str(root / "bench.py"), "--gpus", "2", "--model", "lenet", "--steps",
             "20", "--warmup", "5", "--fused", "1"], cwd=tmp_path,
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-2000:] for o in outs]
    line = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    # on the fallback (gloo all-reduce, host-side) the step cannot be captured
    assert res["n_gpus"] == 2 and res["config"]["hip_graph"] is (corrupt is None)
    assert res["config"]["fused_step"] is True and res["value"] > 0
    assert res["config"]["hip_graph_steps"] == (None if corrupt else 25)
    assert res["replicas_in_sync"] is True
    # the small-bucket path was chosen by the startup self-check (one xGMI call vs the group's
    # all-reduce on the same data, exact); a forced mismatch falls back on both ranks
    assert res["allreduce_selfcheck"] == "pass"
    if corrupt:
        assert res["xgmi_selfcheck"] == "fail" and res["small_allreduce_used"] == "rccl"
    else:
        assert res["xgmi_selfcheck"] == "pass" and res["small_allreduce_used"] == "xgmi"
