"""Headline benchmark: task3 DDP CNN training throughput on 1..8 MI355X.

Metric (BASELINE.json): "samples/sec (whole node) for task3 DDP CNN at 1/2/4/8
MI355X"; the scaling-curve headline config is the ResNet-18-shaped CNN, DDP, bf16.
Batches come through the task3 data path (reference codes/task3/model.py:111-113):
``MySampler`` (random partition, ``set_epoch`` every epoch) over a synthetic dataset
resident on every GPU, drawn by ``DeviceLoader`` (random-init weights, synthetic data;
BASELINE: synthetic data).  Each rank trains on its own shard, so per-GPU work is fixed
as N grows ("weak" scaling).  One timed step = the loader's batch + forward + backward
(with bucketed RCCL all-reduce overlapped) + fused SGD-momentum update of all 11.7 M
parameters.

    python bench.py --gpus 1 --steps 20 --warmup 5          # ResNet-18, 1024 img per GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 ...
    torchrun --nproc-per-node 1 ... bench.py --force-comm 1  # the RCCL path at one rank

``--model lenet`` benchmarks the reference LeNet at the reference batch (32/rank).

At world size > 1 (or with ``--force-comm``) the JSON line also proves the run was what it
claims: ``distinct_gpus`` (device UUIDs gathered from every rank), ``rccl_world`` (the
RCCL communicator's size), ``replicas_in_sync`` (MIN == MAX over ranks of two checksums of
the flat parameters after the timed steps) and ``phases_ms`` (forward / backward compute /
communication left exposed after backward / optimizer, HIP events over a few extra steps).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "samples/sec (whole node) for task3 DDP CNN at 1/2/4/8 MI355X"
# stock PyTorch-ROCm 2.10 (MIOpen/hipBLASLt, channels_last bf16 autocast, SGD) on one
# MI355X at the same per-GPU batch, measured by tools/probe_stock.py: the best of the
# default run (profiles/stock_pytorch_rocm_r1.jsonl) and the --tuned run with
# cudnn.benchmark = True (MIOpen solver search; LeNet without the per-step loss.item()),
# profiles/stock_pytorch_rocm_tuned_r1s5.jsonl
# (1024: default run only, profiles/stock_pytorch_rocm_b1024_r2c.jsonl; the tuned solver
# search outran gpurun's silence limit)
STOCK_PER_GPU = {("resnet18", 256): 16912.7, ("resnet18", 512): 19785.8,
                 ("resnet18", 1024): 18581.2, ("lenet", 32): 49523.7}
# the ratio is quoted against stock's BEST measured per-GPU configuration of the model (not
# the same-batch entry, which mixes tuned and untuned runs): ResNet-18 tuned at 512 images,
# LeNet at the reference batch 32
STOCK_BEST = {"resnet18": (19785.8, "tuned MIOpen, 512 img/GPU"), "lenet": (49523.7, "batch 32")}
# per-GPU batch of the headline run: 1024 images.  A ~1.3 ms/step fixed cost (BN statistic
# reductions, weight-gradient slab reduces, optimizer, launch floor) is amortised over more
# work: 256 -> 36.7k, 512 -> 44.5k, 768 -> 46.5k, 1024 -> 46.7-46.9k img/s on one MI355X
# (profiles/batch_sweep_r2c.jsonl); twice the 512-image activations, a small part of the
# 288 GB HBM3E.  The native step matches stock PyTorch's loss at this batch
# (profiles/batch_numerics_r2c.jsonl).
RESNET_BATCH = 1024


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet18", choices=["resnet18", "lenet"])
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch")
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--dtype", default=None, choices=["fp32", "bf16"],
                    help="activation dtype; default bf16 for resnet18 (always), fp32 for "
                         "lenet (the reference dtype; bf16 = BASELINE config 3)")
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--phases", type=int, default=-1,
                    help="after the timed run, N extra eager steps timed per phase with HIP "
                         "events (fwd, bwd compute, exposed comm, optimizer) -> 'phases_ms'; "
                         "-1 = auto (5 on the native backend)")
    ap.add_argument("--small-allreduce", default="auto", choices=["auto", "rccl", "xgmi"],
                    help="buckets <= 4 MB via the one-shot xGMI peer-memory kernel.  auto: "
                         "LeNet (207 KB of gradients, SURVEY 2.4's design point) uses it when "
                         "the startup self-check (one xGMI call vs RCCL, exact) passes on every "
                         "rank, else RCCL; ResNet-18 (25 MB buckets) always RCCL.  xgmi: the "
                         "same self-check, RCCL on failure")
    ap.add_argument("--xgmi-cap-mb", type=float, default=4.0,
                    help="largest bucket sent through the xGMI kernel with --small-allreduce "
                         "xgmi; above the bucket size every bucket goes there (two-shot)")
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--backend", default="native", choices=["native", "torch"])
    ap.add_argument("--force-comm", type=int, default=0,
                    help="at one rank: initialise a 1-rank RCCL group and run DDP's full "
                         "communication path anyway (reducer, bucket hooks, every bucket's "
                         "all-reduce, buffer broadcasts) -- the multi-GPU code on one GPU")
    ap.add_argument("--init-pg", type=int, default=0,
                    help="diagnostic: at one rank, initialise the 1-rank RCCL process group but "
                         "train without communication (isolates the cost of RCCL's presence "
                         "from that of the DDP communication path)")
    ap.add_argument("--buffer-sync-every", type=int, default=1,
                    help="DDP broadcast_buffers period in training forwards (1 = every step, "
                         "as torch DDP; 0 = never)")
    ap.add_argument("--data", default="loader", choices=["loader", "resident"],
                    help="loader: MySampler + DeviceLoader over a device-resident synthetic "
                         "dataset (the task3 data path); resident: two fixed batches per rank")
    ap.add_argument("--dataset-batches", type=int, default=2,
                    help="ResNet-18: dataset size in per-rank batches (x world size images, "
                         "held on every GPU)")
    ap.add_argument("--stream-priority", default="high", choices=["normal", "high"],
                    help="high (default): run the step on a high-priority stream "
                         "(dmlab.utils.streams): the critical path gets workgroups ahead of the "
                         "weight-gradient stream; +1.3 %% on one MI355X, 51.1-51.5k vs 50.5-50.7k "
                         "img/s interleaved (profiles/stream_priority_ab_r4d.txt)")
    ap.add_argument("--pg-timeout", type=float, default=120.0,
                    help="process-group timeout (s): a hung collective fails the run fast")
    ap.add_argument("--fused", type=int, default=-1,
                    help="LeNet: the whole training step as 2 native dispatches "
                         "(dmlab.models.lenet_fused; 3 + the all-reduce with DDP); -1 = auto (on "
                         "for the native backend)")
    ap.add_argument("--graph-steps", type=int, default=25,
                    help="fused LeNet with --graph: training steps per captured graph (each one "
                         "a complete step through the device cursor; the epoch's last steps "
                         "and a remainder of --steps replay the 1-step graph; capped at "
                         "--steps). The timed region runs exactly --steps steps.  25 divides the "
                         "1875-batch epoch: 1.035M vs 0.897M img/s at 1 step per graph "
                         "(profiles/bench_lenet_graph_steps_ab_r4az.txt)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the whole step (fwd+bwd+all-reduce+opt) in a hipGraph; "
                         "-1 = auto: on for the launch-bound LeNet at any world size (RCCL "
                         "collectives are captured with the step; gloo cannot be); off for "
                         "ResNet-18, whose step is GPU-bound and whose weight gradients run "
                         "on a second stream (eager two-stream 39.4k img/s vs 38.2-38.4k "
                         "captured, one MI355X, profiles/wgrad_stream_ab_r1s4.txt)")
    return ap.parse_args()


def build_data(a, dev, rank, ws, bs):
    """Device-resident synthetic dataset + MySampler (random partition) + DeviceLoader."""
    from dmlab.data import DeviceLoader, MySampler, SyntheticImageNet, TensorDataset

    if a.model == "resnet18":
        n = bs * ws * max(1, a.dataset_batches)
        # every rank generates the same dataset (seed 0) in place on its GPU; the sampler
        # hands each rank a disjoint shard of it per epoch
        ds = SyntheticImageNet(n, a.res, 1000, device=dev, seed=0)
    else:
        from dmlab.data import SyntheticMNIST

        act = torch.bfloat16 if a.dtype == "bf16" else torch.float32
        m = SyntheticMNIST(train=True)  # the 60k-sample MNIST-shaped training set
        ds = TensorDataset(m.images.to(dev, act), m.labels.to(dev))
    sampler = MySampler(ds, ws, rank, shuffle=True, seed=0, mode="partition")
    return DeviceLoader(ds, bs, sampler=sampler, drop_last=True)


def main():
    a = parse()
    # keep stdout to the one JSON line: RCCL's version banner goes to stdout otherwise
    if os.environ.get("NCCL_DEBUG", "VERSION") == "VERSION":
        os.environ["NCCL_DEBUG"] = "WARN"
    import dmlab  # noqa: F401  (HIP hardware-queue count, before the runtime initialises)
    from dmlab.models import Net, ResNet18
    from dmlab.nn import cross_entropy
    from dmlab.optim import SGD
    from dmlab.parallel import DDP, env

    ws_env = int(os.environ.get("WORLD_SIZE", "1"))
    if ws_env > 1 or a.force_comm or a.init_pg:
        dev = env.init(timeout_s=a.pg_timeout,
                       backend="nccl" if ((a.force_comm or a.init_pg) and ws_env == 1) else None)
    else:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
    rank, ws = env.get_rank(), env.get_world_size()
    if a.gpus != ws:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
    comm = ws > 1 or bool(a.force_comm)

    # device-path self-checks before anything is built or timed (dmlab.parallel.selfcheck):
    # RCCL's all-reduce against a closed-form sum, and for LeNet the xGMI small-bucket kernel
    # against RCCL; every rank takes the same path
    checks = {}
    if comm:
        from dmlab.parallel import selfcheck

        checks.update(selfcheck.allreduce_selfcheck(dev))
        if checks["allreduce_selfcheck"] != "pass":
            print(json.dumps({"error": "all-reduce self-check failed", **checks}), flush=True)
            raise SystemExit(3)
        # auto: LeNet only (its 207 KB of gradients are the one-shot kernel's design point);
        # an explicit --small-allreduce xgmi runs the same self-check for any model
        want_xgmi = (a.small_allreduce == "xgmi"
                     or (a.small_allreduce == "auto" and a.model == "lenet"))
        if want_xgmi and dev.type == "cuda":
            checks.update(selfcheck.xgmi_selfcheck(dev))
        else:
            checks.update(xgmi_selfcheck="skipped", small_allreduce_used="rccl")
        a.small_allreduce = checks["small_allreduce_used"]
    elif a.small_allreduce == "auto":
        a.small_allreduce = "rccl"

    torch.manual_seed(0)
    if a.model == "resnet18":
        bs = a.batch or RESNET_BATCH
        model = ResNet18(num_classes=1000).to(dev)
        lr = 0.1
    else:
        bs = a.batch or 32
        model = Net().to(dev)
        lr = 0.001
    if a.backend == "torch":
        model.set_backend("torch")
    opt = SGD(model.parameters(), lr=lr, momentum=0.9)
    net = DDP(model, bucket_cap_mb=a.bucket_mb,
              comm_dtype=torch.bfloat16 if a.comm_dtype == "bf16" else None,
              small_allreduce="xgmi" if a.small_allreduce == "xgmi" else None,
              small_cap_mb=a.xgmi_cap_mb, force_comm=bool(a.force_comm),
              broadcast_buffers=a.buffer_sync_every > 0,
              buffer_sync_every=max(1, a.buffer_sync_every))
    net.fold_average_into(opt)
    if a.fused < 0:
        # the 2-dispatch fused step: 587k vs 205k img/s layer-wise at batch 32
        # (profiles/bench_lenet_fused_v2_r3b.jsonl)
        a.fused = 1 if (a.model == "lenet" and a.backend == "native") else 0
    fused = None
    if a.fused and a.model == "lenet":
        from dmlab.models.lenet_fused import FusedLeNetStep

        fused = FusedLeNetStep(model, opt, ddp=net)

    if a.data == "loader":
        loader = build_data(a, dev, rank, ws, bs)
        data_desc = (f"synthetic {'ImageNet' if a.model == 'resnet18' else 'MNIST'}-shaped "
                     f"dataset of {len(loader.dataset)} samples resident on each GPU, "
                     "MySampler(random partition, set_epoch) + DeviceLoader; random-init weights")
    else:
        loader = None
        data_desc = "synthetic (two device-resident random batches per rank, random-init weights)"
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        if a.model == "resnet18":
            pool = [torch.rand(bs, 3, a.res, a.res, device=dev, generator=g)
                    .contiguous(memory_format=torch.channels_last) for _ in range(2)]
            labels = [torch.randint(0, 1000, (bs,), device=dev, generator=g) for _ in range(2)]
        else:
            act = torch.bfloat16 if a.dtype == "bf16" else torch.float32
            pool = [torch.rand(bs, 1, 28, 28, device=dev, generator=g).to(act) for _ in range(2)]
            labels = [torch.randint(0, 10, (bs,), device=dev, generator=g) for _ in range(2)]

    def train_step(x, y, cursor=None):
        if fused is not None:
            return fused(x, y, cursor=cursor)
        if a.backend == "torch":
            if not isinstance(x, torch.Tensor):
                x = x.materialize()
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.model == "resnet18"):
                out = net(x)
            loss = torch.nn.functional.cross_entropy(out.float(), y)
        else:
            loss = cross_entropy(net(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss.detach()

    if a.graph < 0:
        # RCCL collectives and the xGMI all-reduce kernel capture with the step; gloo's
        # host-side collectives cannot (LeNet's 207 KB of gradients fit one xGMI bucket)
        capturable_comm = (not comm or dist.get_backend() == "nccl"
                           or a.small_allreduce == "xgmi")
        a.graph = 1 if (a.model == "lenet" and capturable_comm) else 0
    a.graph = bool(a.graph and a.backend == "native")

    # ------------------------------------------------------------------ step sources
    batches = None

    def step_reset():
        pass
    if a.graph:
        from dmlab.utils.graph import CapturedStep

        if loader is not None and fused is not None:
            # the epoch order lives on the device; the captured fused step gathers its
            # samples through it and advances the cursor itself (no per-step host work)
            cur = loader.cursor()
            ds = loader.dataset
            # the captures' eager warm-up steps are not part of the run: snapshot the weights,
            # the momentum buffer and the step counter, restore them in place afterwards (as
            # dmlab.tasks.common.train_fused does), so every --graph-steps value trains the
            # same step sequence from the same state
            flat = model.flat
            buf = getattr(opt, "buf", None)
            saved = (flat.data.clone(), buf.clone() if buf is not None else None,
                     getattr(opt, "step_count", 0))
            if getattr(opt, "step_count", 0) == 0:
                opt.step_count = 1  # capture the not-first-step update: buf = m*0 + g = g
            cap = CapturedStep(lambda x, y: train_step(x, y, cursor=cur),
                               [ds.images, ds.labels], warmup=3, bind_inputs=True)
            # a k-step replay never runs past the steps the caller asked for: the timed
            # region executes EXACTLY --steps training steps (k = min(graph-steps, steps))
            kg = max(1, min(a.graph_steps, a.steps))
            capk = None
            if kg > 1:
                def multi(x, y):
                    for _ in range(kg):
                        out = train_step(x, y, cursor=cur)
                    return out

                cur.refill(0)
                capk = CapturedStep(multi, [ds.images, ds.labels], warmup=1, bind_inputs=True)
            # credit: steps a k-step replay already ran ahead of the caller's step count
            state = {"step": 0, "epoch": 0, "credit": 0, "out": None, "budget": a.warmup}

            def step(i):
                if state["credit"]:
                    state["credit"] -= 1
                    return state["out"]
                if state["step"] and state["step"] % cur.nbatch == 0:
                    state["epoch"] += 1
                    cur.refill(state["epoch"])  # next epoch's shard order, same buffer
                left = cur.nbatch - state["step"] % cur.nbatch
                if capk is not None and left >= kg and state["budget"] >= kg:
                    state["out"], n = capk(ds.images, ds.labels), kg
                else:
                    state["out"], n = cap(ds.images, ds.labels), 1
                state["step"] += n
                state["budget"] -= n
                state["credit"] = n - 1
                return state["out"]

            def step_reset():  # the timed region starts on a fresh replay
                state["credit"] = 0
                state["budget"] = a.steps

            with torch.no_grad():
                flat.data.copy_(saved[0])
                flat.mark_updated()
                if buf is not None:
                    buf.copy_(saved[1])
            opt.step_count = saved[2]
            # restart the epoch after the capture warm-up advanced the cursor
            cur.refill(0)
        else:
            if loader is not None:  # layer-wise LeNet: one graph per resident batch slot
                it = iter(loader)
                pool_g, labels_g = zip(*[next(it) for _ in range(2)])
                pool, labels = [t.clone() for t in pool_g], [t.clone() for t in labels_g]
            captured = [CapturedStep(train_step, [pool[k], labels[k]], warmup=3, bind_inputs=True)
                        for k in range(2)]

            def step(i):
                if loader is not None:
                    x, y = next_batch()
                    pool[i % 2].copy_(x, non_blocking=True)
                    labels[i % 2].copy_(y, non_blocking=True)
                return captured[i % 2](pool[i % 2], labels[i % 2])
    else:
        def step(i):
            if loader is None:
                return train_step(pool[i % 2], labels[i % 2])
            x, y = next_batch()
            return train_step(x, y)

    epoch_state = {"epoch": 0, "it": None}

    def next_batch():
        while True:
            if epoch_state["it"] is None:
                loader.set_epoch(epoch_state["epoch"])
                epoch_state["it"] = (loader.iter_gathered() if a.model == "resnet18"
                                     else iter(loader))
            try:
                return next(epoch_state["it"])
            except StopIteration:
                epoch_state["it"] = None
                epoch_state["epoch"] += 1

    run_ctx = contextlib.nullcontext()
    if a.stream_priority == "high":
        from dmlab.utils.streams import compute_stream

        cs = compute_stream(dev)
        cs.wait_stream(torch.cuda.current_stream())
        run_ctx = torch.cuda.stream(cs)
    with run_ctx:
        for i in range(a.warmup):
            loss = step(i)
        step_reset()
        torch.cuda.synchronize()
        env.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            loss = step(i)
        torch.cuda.synchronize()
        env.barrier()
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    final_loss = float(loss)
    # checksum of the flat fp32 parameters after the timed steps (float64 sums): equal bits
    # give equal values, so two runs of the same step sequence can be compared exactly
    pflat = model.flat.data if getattr(model, "flat", None) is not None else torch.cat(
        [p.detach().reshape(-1) for p in model.parameters()])
    pw = (torch.arange(pflat.numel(), device=pflat.device, dtype=torch.float64) % 251) + 1.0
    param_checksum = [float(pflat.double().sum()), float((pflat.double() * pw).sum())]
    verify = verify_replicas(model, dev) if comm else None
    if a.phases < 0:
        a.phases = 5 if a.backend == "native" else 0
    phases = None
    if a.phases > 0 and a.backend == "native":
        if loader is not None:
            src = [next_batch() for _ in range(2)]
        else:
            src = list(zip(pool, labels))
        phases = measure_phases(net, opt, src, a.phases)
    ms = dt / a.steps * 1e3
    value = bs * ws * a.steps / dt
    if rank == 0:
        if comm:
            ddp_desc = (f"bucketed all-reduce overlapped with backward, {len(net.buckets)} buckets "
                        f"(cap {a.bucket_mb} MB), comm {a.comm_dtype}, "
                        f"{'xGMI kernel <= ' + str(a.xgmi_cap_mb) + ' MB, ' if net._xgmi else ''}"
                        f"{'native C++ reducer' if net._native is not None else 'python reducer'}"
                        + (" (forced at one rank)" if ws == 1 else ""))
        else:
            ddp_desc = "none (dp1: no communication)"
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": ws,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "vs_stock_pytorch_rocm": (round(value / (STOCK_BEST[a.model][0] * ws), 3)
                                      if not (a.model == "lenet" and a.dtype == "bf16")
                                      else None),
            "stock_reference": f"stock PyTorch-ROCm best measured: {STOCK_BEST[a.model][1]}",
            "dtype": "bf16" if (a.model == "resnet18" or a.dtype == "bf16") else "fp32",
            "data": data_desc,
            "config": {
                "model": a.model,
                "global_batch": bs * ws,
                "per_gpu_batch": bs,
                "seq_len": None,
                "image_size": a.res if a.model == "resnet18" else 28,
                "parallelism": f"dp{ws}",
                "optimizer": "SGD(momentum=0.9), fused flat",
                "ddp": ddp_desc,
                "process_group": (dist.get_backend() if env.is_initialized() else None),
                "backend": a.backend,
                "fused_step": bool(fused is not None),
                "ddp_side_stream_hooks": (net.side_stream_hooks if comm else None),
                "ddp_buffer_sync_every": (a.buffer_sync_every if comm else None),
                "hip_graph": a.graph,
                "hip_graph_steps": (max(1, a.graph_steps) if (a.graph and fused is not None
                                                            and loader is not None) else None),
                "stream_priority": a.stream_priority,
                "sampler": ("MySampler(partition)" if loader is not None else None),
            },
            "final_loss": round(final_loss, 4),
            "param_checksum": param_checksum,
            "peak_mem_gb": round(torch.cuda.max_memory_reserved() / 2**30, 1),
            "peak_alloc_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1),
            # allocator retries (a failed hipMalloc frees the cache and synchronises): >0
            # means the step ran short of device memory
            "alloc_retries": int(torch.cuda.memory_stats().get("num_alloc_retries", 0)),
        }
        if verify is not None:
            res.update(verify)
        res.update(checks)
        if comm:
            res["buckets_launched"] = int(net.buckets_launched)
        if phases is not None:
            res["phases_ms"] = phases
        print(json.dumps(res), flush=True)
    env.destroy()


def verify_replicas(model, dev):
    """Multi-rank self-check: which GPUs the ranks ran on, the communicator size, and whether
    every replica holds the same parameters after the timed steps (MIN == MAX over ranks of
    two checksums of the flat fp32 parameters; identical bits give identical checksums)."""
    from dmlab.parallel.xgmi import _device_key

    keys = [None] * dist.get_world_size()
    dist.all_gather_object(keys, _device_key(dev) if dev.type == "cuda" else "cpu")
    flat = model.flat.data if getattr(model, "flat", None) is not None else torch.cat(
        [p.detach().reshape(-1) for p in model.parameters()])
    x = flat.double()
    w = (torch.arange(x.numel(), device=x.device, dtype=torch.float64) % 251) + 1.0
    ck = torch.stack([x.sum(), (x * w).sum()])
    lo, hi = ck.clone(), ck.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    diff = float((hi - lo).abs().max())
    return {
        "distinct_gpus": len(set(keys)),
        "rccl_world": dist.get_world_size() if dist.get_backend() == "nccl" else None,
        "replicas_in_sync": bool(torch.equal(lo, hi)),
        "replica_checksum_spread": diff,
    }


def measure_phases(net, opt, src, n):
    """Per-phase device time of n eager steps (HIP events, one sync at the end):
    forward+loss, backward compute, communication still outstanding when backward
    compute ends (exposed), optimizer."""
    from dmlab.nn import cross_entropy

    names = ("fwd", "bwd_compute", "comm_exposed", "opt")
    acc = {k: 0.0 for k in names}
    for i in range(n):
        x, y = src[i % len(src)]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        net.on_compute_done = ev[2].record
        ev[0].record()
        loss = cross_entropy(net(x), y)
        ev[1].record()
        opt.zero_grad()
        loss.backward()
        ev[3].record()
        opt.step()
        ev[4].record()
        net.on_compute_done = None
        torch.cuda.synchronize()
        for k, (a_, b_) in zip(names, ((0, 1), (1, 2), (2, 3), (3, 4))):
            acc[k] += ev[a_].elapsed_time(ev[b_])
    return {k: round(v / n, 3) for k, v in acc.items()}


if __name__ == "__main__":
    main()
