"""All-reduce latency/bandwidth sweep: RCCL vs the xGMI peer-memory kernels.

One process per GPU (torchrun), fp32 messages from 4 KB to 64 MB, each timed with HIP
events over ``--iters`` back-to-back calls; rank 0 prints one JSON line per size with the
per-call time and the bus bandwidth 2(W-1)/W * bytes / t of each algorithm:

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py

``DMLAB_BACKEND=gloo`` (ranks sharing one GPU, as on a one-GPU box) skips the RCCL column
and only checks and times the peer-memory kernels -- there all ranks share one HBM, so
the numbers say nothing about xGMI; they are a functional rehearsal.
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dmlab.parallel import env  # noqa: E402
from dmlab.parallel.xgmi import XGMIAllReduce  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    env.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    t = torch.tensor([e0.elapsed_time(e1) / iters], device="cuda")
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    else:
        t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t) * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--min-kb", type=int, default=4)
    ap.add_argument("--max-mb", type=int, default=64)
    a = ap.parse_args()
    dev = env.init()
    rank, W = env.get_rank(), env.get_world_size()
    sizes = []
    b = a.min_kb * 1024
    while b <= a.max_mb * 2**20:
        sizes.append(b // 4)
        b *= 4
    xg = XGMIAllReduce(cap=max(sizes), device=dev)
    rccl = dist.get_backend() == "nccl"
    for n in sizes:
        t = torch.full((n,), float(rank + 1), device=dev)
        row = {"bytes": n * 4, "world": W}
        bus = 2 * (W - 1) / W * n * 4
        for name in ("one_shot", "two_shot"):
            # correctness first: sum of (rank + 1) over ranks
            x = torch.full((n,), float(rank + 1), device=dev)
            xg(x, algo=name)
            ok = bool((x == W * (W + 1) / 2).all())
            sec = timed(lambda: xg(t.fill_(1.0), algo=name), a.iters)
            row[name] = {"us": round(sec * 1e6, 2), "busbw_GBs": round(bus / sec / 1e9, 1), "ok": ok}
        if rccl:
            sec = timed(lambda: dist.all_reduce(t), a.iters)
            row["rccl"] = {"us": round(sec * 1e6, 2), "busbw_GBs": round(bus / sec / 1e9, 1)}
        xg.check()
        if rank == 0:
            print(json.dumps(row), flush=True)
    xg.close()
    env.destroy()


if __name__ == "__main__":
    main()
