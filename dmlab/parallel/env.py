"""Process-group bring-up: torchrun env:// or the reference's explicit CLI.

Reference: ``dist_init(world_size, rank, master_addr, master_port)`` sets
MASTER_ADDR/PORT and calls ``init_process_group("nccl")`` (task2/dist_utils.py:6-15;
task4/dist_utils.py:12 uses gloo).  ``get_local_rank`` there returns the *global*
rank; here global and node-local rank are distinct.

MI355X design: one process per GPU; ``LOCAL_RANK`` selects the device (the
reference pins every spawned rank to GPU 0, B5); backend ``"nccl"`` is RCCL over
xGMI on ROCm, ``"gloo"`` for CPU runs and tests.  The process group is created
with ``device_id`` so RCCL communicators initialise eagerly and bind to the
right GPU.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

_DEVICE = None


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_rank() -> int:
    return dist.get_rank() if is_initialized() else int(os.environ.get("RANK", 0))


def get_world_size() -> int:
    return dist.get_world_size() if is_initialized() else int(os.environ.get("WORLD_SIZE", 1))


def get_local_rank() -> int:
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    if is_initialized():
        n = torch.cuda.device_count() if torch.cuda.is_available() else 0
        return get_rank() % n if n else get_rank()
    return 0


def get_local_world_size() -> int:
    return int(os.environ.get("LOCAL_WORLD_SIZE", get_world_size()))


def default_backend(device: torch.device | str | None = None) -> str:
    if device is not None:
        return "nccl" if torch.device(device).type == "cuda" else "gloo"
    return "nccl" if torch.cuda.is_available() else "gloo"


def device() -> torch.device:
    global _DEVICE
    if _DEVICE is None:
        if torch.cuda.is_available() and os.environ.get("DMLAB_DEVICE", "cuda") != "cpu":
            _DEVICE = torch.device("cuda", get_local_rank() % max(torch.cuda.device_count(), 1))
        else:
            _DEVICE = torch.device("cpu")
    return _DEVICE


def init(world_size: int | None = None, rank: int | None = None, master_addr: str | None = None,
         master_port: str | int | None = None, backend: str | None = None,
         device_type: str | None = None, timeout_s: float = 600.0) -> torch.device:
    """Initialise the default process group and bind this process to its device.

    torchrun/env variables take precedence; explicit arguments reproduce the
    reference CLI (``--n_devices --rank --master_addr --master_port``)."""
    global _DEVICE
    env_ws = os.environ.get("WORLD_SIZE")
    ws = int(env_ws) if env_ws is not None else (world_size or 1)
    rk = int(os.environ["RANK"]) if "RANK" in os.environ else (rank or 0)
    if master_addr is not None and "MASTER_ADDR" not in os.environ:
        os.environ["MASTER_ADDR"] = str(master_addr)
    if master_port is not None and "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(master_port)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "12355")
    if device_type is None:
        # DMLAB_DEVICE=cpu (set by ``dmlab.launch --cpu``) forces gloo/CPU ranks
        device_type = os.environ.get("DMLAB_DEVICE") or (
            "cuda" if torch.cuda.is_available() else "cpu")
    if device_type == "cuda":
        ndev = max(torch.cuda.device_count(), 1)
        # more local ranks than GPUs: ranks share devices round-robin (only usable with
        # gloo, DMLAB_BACKEND=gloo -- RCCL rejects two ranks on one GPU, loudly)
        lr = int(os.environ.get("LOCAL_RANK", rk)) % ndev
        _DEVICE = torch.device("cuda", lr)
        torch.cuda.set_device(_DEVICE)
    else:
        _DEVICE = torch.device("cpu")
        # CPU ranks share the host: split the cores instead of oversubscribing
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", ws))
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // max(lws, 1)))
    # DMLAB_BACKEND overrides the choice (e.g. gloo for GPU ranks that share one device in
    # tests: RCCL refuses two ranks on the same GPU)
    backend = backend or os.environ.get("DMLAB_BACKEND") or default_backend(_DEVICE)
    if ws > 1 or backend is not None:
        if not is_initialized():
            kw = dict(backend=backend, rank=rk, world_size=ws,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = _DEVICE
                # RCCL on a high-priority stream: the training step's critical path already
                # runs at high priority (dmlab.utils.streams), and the bucket all-reduces must
                # keep progressing next to it rather than queue behind the weight gradients
                opts = getattr(dist, "ProcessGroupNCCL", None)
                if (opts is not None and hasattr(opts, "Options")
                        and os.environ.get("DMLAB_PG_HIGH_PRIORITY", "1") != "0"):
                    o = opts.Options()
                    o.is_high_priority_stream = True
                    kw["pg_options"] = o
            dist.init_process_group(**kw)
        assert dist.is_initialized(), "Error! The distributed env is not initialized!"
    return _DEVICE


def destroy():
    if is_initialized():
        dist.destroy_process_group()


def barrier():
    if is_initialized() and get_world_size() > 1:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device().index])
        else:
            dist.barrier()
