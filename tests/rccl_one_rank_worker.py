"""Worker for tests/test_rccl_gpu.py: one scenario per process, under a 1-RANK RCCL
(ProcessGroupNCCL) communicator on the box's single GPU.  RCCL accepts a 1-rank
communicator, so every collective the multi-GPU path issues -- the native reducer's
``pg->allreduce`` per bucket from the side-stream hooks, bf16 gradient communication,
``broadcast_buffers``, ``init_parameters``, RCCL inside a captured hipGraph -- executes here
exactly as it does at eight ranks (minus the link traffic).

Prints one JSON line ``{"scenario": ..., "ok": bool, ...}``.
"""
import json
import os
import sys
import traceback
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _grads_resnet(ddp_kw, force):
    from dmlab.models import ResNet18
    from dmlab.nn import cross_entropy
    from dmlab.optim import SGD
    from dmlab.parallel import DDP

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    X = torch.rand(8, 3, 64, 64, generator=g).to(dev)
    Y = torch.randint(0, 10, (8,), generator=g).to(dev)
    torch.manual_seed(0)
    model = ResNet18(num_classes=10).to(dev)
    ddp = DDP(model, force_comm=force, **ddp_kw)
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9)
    ddp.fold_average_into(opt)
    grads = []
    for _ in range(2):
        opt.zero_grad()
        cross_entropy(ddp(X), Y).backward()
        grads.append(model.flat.grad.clone())
        opt.step()
    torch.cuda.synchronize()
    return ddp, grads, model.flat.data.clone()


def scenario_resnet_fp32():
    """(a) ResNet-18 DDP, side-stream bucket hooks, fp32 RCCL all-reduce of every bucket ==
    the no-communication run, bit for bit (SUM over one rank is the identity)."""
    ddp, g1, p1 = _grads_resnet({}, True)
    assert ddp._native is not None and ddp.side_stream_hooks
    launched = ddp.buckets_launched
    nb = len(ddp.buckets)
    _, g0, p0 = _grads_resnet({}, False)
    return dict(ok=all(torch.equal(a, b) for a, b in zip(g1, g0)) and torch.equal(p1, p0),
                buckets=nb, launched=launched, expect_launched=2 * nb,
                max_diff=max(float((a - b).abs().max()) for a, b in zip(g1, g0)))


def scenario_resnet_bf16():
    """(a) bf16 gradient communication through the persistent comm buffer: the reduced
    gradient is exactly the bf16 rounding of the local one (first step; same init)."""
    ddp, g1, _ = _grads_resnet({"comm_dtype": torch.bfloat16}, True)
    assert ddp._comm_flat is not None and ddp.side_stream_hooks
    _, g0, _ = _grads_resnet({}, False)
    want = g0[0].to(torch.bfloat16).float()
    return dict(ok=torch.equal(g1[0], want), launched=ddp.buckets_launched,
                max_diff=float((g1[0] - want).abs().max()))


def scenario_lenet_graph():
    """(b) the fused LeNet DDP step with the RCCL all-reduce captured in a hipGraph, replayed,
    == the same step run eagerly (bit for bit)."""
    from dmlab.models import Net
    from dmlab.models.lenet_fused import FusedLeNetStep
    from dmlab.optim import SGD
    from dmlab.parallel import DDP
    from dmlab.utils.graph import CapturedStep

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    X = torch.rand(32, 1, 28, 28, generator=g).to(dev)
    Y = torch.randint(0, 10, (32,), generator=g).to(dev)
    runs = []
    for captured in (False, True):
        torch.manual_seed(0)
        model = Net().to(dev)
        ddp = DDP(model, force_comm=True)
        assert ddp._native is not None
        opt = ddp.fold_average_into(SGD(model.parameters(), lr=0.1, momentum=0.9))
        step = FusedLeNetStep(model, opt, ddp=ddp)
        assert not step._fused_sgd()  # the all-reduce sits between gradients and SGD
        if captured:
            cap = CapturedStep(step, [X, Y], warmup=2, bind_inputs=True)
            for _ in range(4):
                cap(X, Y)
        else:
            for _ in range(6):
                step(X, Y)
        torch.cuda.synchronize()
        runs.append((model.flat.data.clone(), ddp.buckets_launched))
    return dict(ok=torch.equal(runs[0][0], runs[1][0]),
                max_diff=float((runs[0][0] - runs[1][0]).abs().max()),
                eager_launched=runs[0][1], graph_launched=runs[1][1])


def scenario_buffers():
    """(c) init_parameters and broadcast_buffers over RCCL: values unchanged (one rank), one
    coalesced broadcast per training forward, and the wrapper is a usable nn.Module
    (state_dict / to)."""
    from dmlab.models import ResNet18
    from dmlab.nn import cross_entropy
    from dmlab.parallel import DDP, comm

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = ResNet18(num_classes=10).to(dev)
    before = model.flat.data.clone()
    comm.init_parameters(model, force=True)
    same = torch.equal(before, model.flat.data)
    ddp = DDP(model, force_comm=True)
    rm = model.stem.running_mean.clone()
    x = torch.rand(4, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (4,), device=dev)
    cross_entropy(ddp(x), y).backward()
    ddp.sync_buffers()
    torch.cuda.synchronize()
    moved = not torch.equal(rm, model.stem.running_mean)  # the forward updated the stats
    sd = ddp.state_dict()
    ddp.to(dev)
    return dict(ok=same and moved and len(sd) > 0 and ddp._fwd_count == 1,
                state_dict_keys=len(sd), bufs=len(ddp._bcast_bufs))


def scenario_p2p_self():
    """(d) stage-to-stage RCCL send/recv to self is unsupported: PGTransport says so."""
    from dmlab.parallel.p2p import PGTransport

    try:
        PGTransport()
    except RuntimeError as e:
        return dict(ok="needs >= 2 ranks" in str(e), msg=str(e))
    return dict(ok=False, msg="no error")


def scenario_aggregator():
    """GradAggregator over RCCL at one rank (forced): all-reduce and all-gather averaging
    leave the gradient unchanged and report device-side communication time."""
    from dmlab.models import Net
    from dmlab.nn import cross_entropy
    from dmlab.parallel import comm

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = Net().to(dev)
    x = torch.rand(16, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (16,), device=dev)
    cross_entropy(model(x), y).backward()
    g0 = model.flat.grad.clone()
    ok = True
    for method in ("allreduce", "allgather"):
        agg = comm.GradAggregator(model, method, force=True)
        for _ in range(3):
            agg()
        ok &= torch.allclose(model.flat.grad, g0) and agg.comm_time > 0
    return dict(ok=bool(ok))


def main():
    name = sys.argv[1]
    from dmlab.parallel import env

    out = {"scenario": name}
    try:
        env.init(backend="nccl", timeout_s=120)
        assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
        out.update(globals()["scenario_" + name]())
    except Exception:
        out.update(ok=False, error=traceback.format_exc())
    finally:
        try:
            env.destroy()
        except Exception:
            pass
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    main()
