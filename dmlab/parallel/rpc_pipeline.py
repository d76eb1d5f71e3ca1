"""RPC/RRef model-parallel facade — the reference lab-4 programming model.

Reference: codes/task4/model.py:49-66 (``ParallelNet`` with ``rpc.remote`` stages
and ``parameter_rrefs``), :68-87 (``dist_autograd.context`` → forward →
``dist_autograd.backward`` → ``DistributedOptimizer.step``), :104-139 (role
dispatch: rank 0 = ``worker0`` driver, ranks 1/2 = passive stage owners).

Kept API-compatible for the lab (same names, same call sequence), with two
deliberate changes:
* stage 1 pulls stage 0's activation *directly* through an RRef (``to_here`` on
  worker2 from worker1) instead of relaying it through the driver;
  ``relay=True`` restores the reference data path;
* the stage modules are dmlab Programs, so on a device they run the native HIP
  kernels and their local optimiser step is the fused flat kernel.

The control plane is torch RPC (TensorPipe).  For GPU stages the data plane of
choice is :mod:`dmlab.parallel.pipeline` (P2P over RCCL/xGMI); TensorPipe device
RPC is beta in PyTorch (sections/task4.tex:26-32), so this facade moves tensors
through the host.
"""
from __future__ import annotations

import torch
import torch.distributed.autograd as dist_autograd
import torch.distributed.rpc as rpc
import torch.nn as nn

from dmlab.models.lenet import SubNetConv, SubNetFC


class RPCStage(nn.Module):
    """A stage module living on its owner worker."""

    def __init__(self, kind: str, arg: int, device: str = "cpu"):
        super().__init__()
        if device == "cuda":  # one GPU per stage owner: worker k -> GPU (k-1) mod #GPUs
            wid = rpc.get_worker_info().id
            device = f"cuda:{(wid - 1) % max(1, torch.cuda.device_count())}"
        self.device = torch.device(device)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.module = (SubNetConv(arg) if kind == "conv" else SubNetFC(arg)).to(self.device)

    def forward(self, x):
        flat = getattr(self.module, "flat", None)
        if flat is not None and torch.is_grad_enabled():
            # one forward per training step: the next backward overwrites grads
            flat.mark_grads_consumed()
        out = self.module(x.to(self.device))
        return out.cpu() if self.device.type != "cpu" else out

    def forward_rref(self, x_rref):
        return self.forward(x_rref.to_here())

    def parameter_rrefs(self):
        return [rpc.RRef(p) for p in self.module.parameters()]


class ParallelNet(nn.Module):
    """Driver-side handle of the two remote stages (reference model.py:49-66)."""

    def __init__(self, in_channels=1, num_classes=10, workers=("worker1", "worker2"),
                 devices=("cpu", "cpu"), relay: bool = False):
        super().__init__()
        self.relay = relay
        self.subnet_conv = rpc.remote(workers[0], RPCStage, args=("conv", in_channels, devices[0]))
        self.subnet_fc = rpc.remote(workers[1], RPCStage, args=("fc", num_classes, devices[1]))

    def forward(self, x):
        if self.relay:  # reference path: worker1 -> driver -> worker2
            h = self.subnet_conv.rpc_sync().forward(x)
            return self.subnet_fc.rpc_sync().forward(h)
        h_rref = self.subnet_conv.remote().forward(x)
        return self.subnet_fc.rpc_sync().forward_rref(h_rref)

    def parameter_rrefs(self):
        out = []
        out.extend(self.subnet_conv.rpc_sync().parameter_rrefs())
        out.extend(self.subnet_fc.rpc_sync().parameter_rrefs())
        return out


def make_distributed_optimizer(model: ParallelNet, lr=0.01, momentum=0.0):
    """Remote per-owner optimiser (reference model.py:126).  Uses dmlab's SGD
    (a Python optimiser, so the fused flat kernel runs on each owner)."""
    from torch.distributed.optim import DistributedOptimizer

    from dmlab.optim import SGD

    return DistributedOptimizer(SGD, model.parameter_rrefs(), lr=lr, momentum=momentum)


def train_step(model, opt, loss_fn, inputs, labels):
    """The reference's per-batch body (model.py:75-84)."""
    with dist_autograd.context() as cid:
        out = model(inputs)
        loss = loss_fn(out, labels)
        dist_autograd.backward(cid, [loss])
        opt.step(cid)
    return loss.detach()
