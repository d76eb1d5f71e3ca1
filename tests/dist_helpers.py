"""Spawn a small gloo process group on the CPU (127.0.0.1) for distributed tests."""
import os
import socket
import sys
import traceback
from pathlib import Path

import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, ws, port, fn, args, errq):
    try:
        sys.path.insert(0, str(ROOT))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(ws), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(ws))
        import torch

        torch.set_num_threads(1)
        from dmlab.parallel import env

        env.init(ws, rank, backend="gloo", device_type="cpu")
        fn(rank, ws, *args)
        env.destroy()
    except Exception:
        errq.put((rank, traceback.format_exc()))
        raise


def run_dist(fn, ws, *args):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, ws, port, fn, args, errq)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    if errs:
        raise AssertionError("\n".join(f"rank {r}:\n{t}" for r, t in errs))
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    assert not bad, f"ranks exited with {bad}"
