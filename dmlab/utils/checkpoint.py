"""Checkpoint / resume (absent in the reference; low priority extension).

Rank 0 writes one file holding the model state dict (parameters + BN buffers), the
optimiser state (lr, step count, momentum/Adam moments) and user extras.  Loading is
``torch.load(weights_only=True)`` (tensors and plain containers only), on every rank,
followed by a broadcast from rank 0 so all replicas start bit-identical.
"""
from __future__ import annotations

import os

import torch

from dmlab.parallel import env


def save(path, model, optimizer=None, **extra):
    module = getattr(model, "module", model)
    if env.get_rank() == 0:
        state = {"model": {k: v.detach().cpu() for k, v in module.state_dict().items()},
                 "extra": extra}
        if optimizer is not None:
            state["optimizer"] = {k: (v.detach().cpu() if torch.is_tensor(v) else v)
                                  for k, v in optimizer.state_dict().items()}
        tmp = f"{path}.tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)  # atomic: a crash never leaves a torn checkpoint
    env.barrier()


def load(path, model, optimizer=None, map_location="cpu"):
    module = getattr(model, "module", model)
    state = torch.load(path, map_location=map_location, weights_only=True)
    module.load_state_dict(state["model"])
    if hasattr(module, "flat") and module.flat is not None:
        module.flat.mark_updated()
    if optimizer is not None and "optimizer" in state:
        dev = next(module.parameters()).device
        optimizer.load_state_dict({k: (v.to(dev) if torch.is_tensor(v) else v)
                                   for k, v in state["optimizer"].items()})
    if env.get_world_size() > 1:
        from dmlab.parallel.comm import init_parameters

        init_parameters(module)
    return state.get("extra", {})
