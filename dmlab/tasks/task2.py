"""Lab 2 — communication & gradient aggregation.

Reference: codes/task2/model.py (one process per CLI invocation, bs 32) and
codes/task2/model-mp.py (self-spawning ``mp.spawn``, bs 30, communication-time
measurement, commented straggler ``time.sleep(0.1)`` on rank 1 and commented
all-gather alternative).  Both: ``DistributedSampler``, SGD lr .01 momentum .9,
2 epochs, per-parameter all-reduce + ``/= ws`` after backward.

Launch any of:
    torchrun --nproc-per-node 2 -m dmlab.tasks.task2 --aggregation allgather
    python -m dmlab.tasks.task2 --n_devices 2 --rank 0   (and --rank 1; reference CLI)
    python -m dmlab.tasks.task2 --n_devices 2 --spawn    (model-mp.py behaviour)
Options: ``--aggregation {allreduce,allgather,allgather_ref}``,
``--granularity {flat,per_param}``, ``--straggler-rank R --straggler-delay-ms D
[--straggler-mode host|device]``.
"""
from __future__ import annotations

import argparse
import json
import os

import torch

from dmlab.data import DeviceLoader, PartitionSampler, load_mnist
from dmlab.models import Net
from dmlab.nn import CrossEntropyLoss
from dmlab.optim import SGD
from dmlab.parallel import comm, env
from dmlab.parallel.straggler import Straggler
from dmlab.tasks.common import test, train


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--n_devices", default=1, type=int, help="The distributed world size.")
    p.add_argument("--rank", default=0, type=int, help="The rank of this process.")
    p.add_argument("--gpu", default=None, type=str, help="(reference flag; device = LOCAL_RANK)")
    p.add_argument("--master_addr", default="127.0.0.1", type=str)
    p.add_argument("--master_port", default="12355", type=str)
    p.add_argument("--spawn", action="store_true", help="self-spawn n_devices ranks (model-mp.py)")
    p.add_argument("--device", default=None, choices=[None, "cpu", "cuda"])
    p.add_argument("--backend", default=None, choices=[None, "nccl", "gloo"])
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--epochs", type=int, default=2)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--aggregation", default="allreduce",
                   choices=["allreduce", "allgather", "allgather_ref", "allreduce_xgmi"],
                   help="allreduce_xgmi: the one-shot xGMI peer-memory kernel over the flat "
                        "gradient buffer (GPU ranks of one node)")
    p.add_argument("--force-comm", action="store_true",
                   help="at one rank with a process group (--backend nccl): run the collectives "
                        "anyway, to measure the device communication path on a single GPU")
    p.add_argument("--granularity", default="flat", choices=["flat", "per_param"])
    p.add_argument("--straggler-rank", type=int, default=None)
    p.add_argument("--straggler-delay-ms", type=float, default=100.0)
    p.add_argument("--straggler-mode", default="host", choices=["host", "device"])
    p.add_argument("--data", default="./data")
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--train-samples", type=int, default=None)
    p.add_argument("--max-steps", type=int, default=None)
    p.add_argument("--no-test", action="store_true")
    p.add_argument("--json", default=None, help="write rank-0 stats JSON here")
    return p.parse_args(argv)


def run(a):
    dev = env.init(a.n_devices, a.rank, a.master_addr, a.master_port, backend=a.backend,
                   device_type=a.device)
    rank, ws = env.get_rank(), env.get_world_size()
    torch.manual_seed(1234 + rank)  # different init per rank; init_parameters syncs it
    model = Net(1, 10).to(dev)
    train_set = load_mnist(a.data, True, synthetic=True if a.synthetic else None, n=a.train_samples)
    test_set = load_mnist(a.data, False, synthetic=True if a.synthetic else None)
    sampler = PartitionSampler(train_set, ws, rank)   # DistributedSampler semantics
    loader = DeviceLoader(train_set.to(dev), a.batch_size, sampler=sampler)
    opt = SGD(model.parameters(), lr=a.lr, momentum=a.momentum)
    comm.init_parameters(model)                       # task2/model.py:46
    agg = comm.GradAggregator(model, a.aggregation, a.granularity, force=a.force_comm)
    strag = Straggler(a.straggler_rank, a.straggler_delay_ms, a.straggler_mode)
    stats = train(model, loader, CrossEntropyLoss(), opt, a.epochs, rank=rank, aggregate=agg,
                  straggler=strag, batch_size=a.batch_size, max_steps=a.max_steps)
    print("Training time: {}".format(stats["train_time"]))
    print(f"Total communication time: {agg.comm_time}")
    if not a.no_test and rank == 0:
        stats["accuracy"] = test(model, DeviceLoader(test_set.to(dev), 32))
    stats.update(rank=rank, world_size=ws, aggregation=a.aggregation, granularity=a.granularity,
                 straggler_rank=a.straggler_rank, straggler_ms=strag.injected_ms,
                 samples_per_s=stats["samples"] * ws / stats["train_time"])
    if a.json and rank == 0:
        with open(a.json, "w") as f:
            json.dump(stats, f)
    env.barrier()
    env.destroy()
    return stats


def _spawn_main(rank, a):
    a.rank = rank
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(a.n_devices)
    run(a)


def main(argv=None):
    a = parse_args(argv)
    if a.spawn and "RANK" not in os.environ:
        import torch.multiprocessing as mp

        mp.spawn(_spawn_main, (a,), nprocs=a.n_devices)
        return None
    return run(a)


if __name__ == "__main__":
    main()
