"""Shared training / evaluation loops with the reference console formats.

Formats:
  "Device {r} starts training ..."                         task2/model.py:41
  'Device: %d epoch: %d, iters: %5d, loss: %.3f'          task2/model.py:66
  'epoch: %d, iters: %5d, loss: %.3f'                     task1/pytorch/model.py:60
  "Finished epoch: {e:3d} / {n:3d}"                       task1/pytorch/model.py:62
  "Training Finished!" / "Training time: {s}" / "Total communication time: {s}"
  '\nTest set: Accuracy: {}/{} ({:.2f}%)\n'              task1/pytorch/model.py:79

Differences from the reference loop, on purpose: the running loss stays on the
device and is read back only when printed (B11: the reference calls
``loss.item()`` every iteration), ``sampler.set_epoch`` is called every epoch (B3),
and evaluation counts correct predictions on the device (K26).
"""
from __future__ import annotations

import contextlib
import time

import torch

from dmlab.nn.loss import count_correct


def _step_stream(model):
    """Training runs on a high-priority stream on the GPU (dmlab.utils.streams): the
    critical path's workgroups go ahead of the weight-gradient side stream's."""
    try:
        p = next(model.parameters())
    except (StopIteration, AttributeError):
        return contextlib.nullcontext()
    if not p.is_cuda:
        return contextlib.nullcontext()
    from dmlab.utils.streams import compute_stream

    st = compute_stream(p.device)
    st.wait_stream(torch.cuda.current_stream(p.device))
    return torch.cuda.stream(st)


def train(model, loader, loss_fn, optimizer, num_epochs=2, *, rank=None, aggregate=None,
          straggler=None, log_every=20, writer=None, batch_size=None, max_steps=None,
          print_fn=print, task1_format=False, after_step=None):
    """Generic loop.  ``aggregate()`` runs between backward and step (manual DP,
    lab 2/3); with :class:`~dmlab.parallel.ddp.DistributedDataParallel` it is None
    (the reducer already overlapped communication with backward).  Returns a
    stats dict (losses printed, steps, samples, times)."""
    if rank is not None:
        print_fn("Device {} starts training ...".format(rank))
    elif task1_format:
        print_fn("Start training ...")
    model.train()
    stats = {"losses": [], "steps": 0, "samples": 0, "comm_time": 0.0}
    with _step_stream(model):
        _train_loop(model, loader, loss_fn, optimizer, num_epochs, stats, rank, aggregate,
                    straggler, log_every, writer, batch_size, max_steps, print_fn, task1_format,
                    after_step)
    print_fn("Training Finished!")
    if writer is not None:
        writer.flush()
    return stats


def _train_loop(model, loader, loss_fn, optimizer, num_epochs, stats, rank, aggregate,
                straggler, log_every, writer, batch_size, max_steps, print_fn, task1_format,
                after_step):
    loss_acc = None
    train_cnt = 0
    t0 = time.perf_counter()
    step = 0
    done = False
    for epoch in range(num_epochs):
        if hasattr(loader, "set_epoch"):
            loader.set_epoch(epoch)
        elif hasattr(getattr(loader, "sampler", None), "set_epoch"):
            loader.sampler.set_epoch(epoch)
        for i, (inputs, labels) in enumerate(loader):
            outputs = model(inputs)
            loss = loss_fn(outputs, labels)
            optimizer.zero_grad()
            loss.backward()
            if aggregate is not None:
                stats["comm_time"] += aggregate() or 0.0
            if straggler is not None:
                straggler()
            optimizer.step()
            if after_step is not None:
                after_step(step)
            ld = loss.detach().float()
            loss_acc = ld if loss_acc is None else loss_acc + ld
            stats["samples"] += inputs.shape[0]
            step += 1
            if i % log_every == log_every - 1:
                avg = float(loss_acc) / log_every  # the only host sync in the loop
                loss_acc = None
                stats["losses"].append(avg)
                if writer is not None:
                    writer.add_scalar("Train Loss", avg, step)
                if task1_format:
                    print_fn('epoch: %d, iters: %5d, loss: %.3f' % (epoch + 1, i + 1, avg))
                else:
                    print_fn('Device: %d epoch: %d, iters: %5d, loss: %.3f'
                             % (rank or 0, epoch + 1, i + 1, avg))
                train_cnt += batch_size or inputs.shape[0]
            if max_steps is not None and step >= max_steps:
                done = True
                break
        if task1_format:
            print_fn(f"Finished epoch: {epoch + 1:3d} / {num_epochs:3d}")
        if done:
            break
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    stats["train_time"] = time.perf_counter() - t0
    stats["steps"] = step
    if aggregate is not None and hasattr(aggregate, "comm_time"):
        stats["comm_time"] = aggregate.comm_time  # event-timed aggregators report here


def train_fused(net, loader, optimizer, num_epochs=2, *, ddp=None, rank=None, log_every=20,
                graph=True, graph_steps=20, max_steps=None, print_fn=print, writer=None,
                drop_last=False):
    """The lab-3 loop (codes/task3/model.py:39-64) on the GPU fast path: the reference LeNet
    step as the 2-dispatch fused kernel pair (:class:`~dmlab.models.lenet_fused.
    FusedLeNetStep`; with ``ddp`` the bucket all-reduce sits between them), its samples
    gathered on the device through the sampler's epoch order (:class:`~dmlab.data.
    DeviceCursor`), the whole step captured in a hipGraph (``graph``) and replayed.
    ``graph_steps`` (a divisor of ``log_every``): complete steps per graph replay; blocks
    that would cross the end of the epoch's whole batches or a ``max_steps`` cut run on the
    1-step graph (one replay per step leaves ~5 us of launch latency per ~31 us step:
    profiles/bench_lenet_graph_steps_ab_r4az.txt).  A shard whose size is not a multiple of
    the batch ends each epoch with one eager fused step on its partial last batch, as the
    reference DataLoader (drop_last=False) does; ``drop_last`` skips it.

    Same console output as :func:`train`: the running loss is summed on the device, copied
    to pinned host memory every ``log_every`` steps and printed once the copy has landed
    (no host synchronisation inside the loop); like the reference loop (and :func:`train`)
    the running sum is reset only after a printed line, so an epoch's tail carries into the
    next epoch's first line.  Returns the same stats dict as :func:`train`."""
    from dmlab.models.lenet_fused import FusedLeNetStep

    if rank is not None:
        print_fn("Device {} starts training ...".format(rank))
    net.train()
    kg = graph_steps if (graph and graph_steps > 1 and log_every % graph_steps == 0) else 1
    step_fn = FusedLeNetStep(net, optimizer, ddp=ddp)
    cur = loader.cursor()
    ds = loader.dataset
    tail = 0 if drop_last else cur.tail.numel()
    if graph:
        from dmlab.utils.graph import CapturedStep

        # the capture's eager warm-up steps must not count as training: snapshot the weights,
        # the momentum buffer and the step counter, and restore them in place afterwards (the
        # graphs keep the pointers).  The captured update is the not-first-step form
        # buf = m*buf + grad (dampening 0, the labs' setting): with a fresh zero buffer that
        # IS the first step's buf = grad, and a resumed run keeps its loaded momentum.
        if getattr(optimizer, "dampening", 0.0):
            raise ValueError("graph-captured fused step: SGD dampening != 0 is not supported")
        flat = net.flat
        buf = getattr(optimizer, "buf", None)
        saved = (flat.data.clone(), buf.clone() if buf is not None else None,
                 getattr(optimizer, "step_count", 0))
        if getattr(optimizer, "step_count", 0) == 0:
            optimizer.step_count = 1  # capture the not-first-step update (see above)
        runner = CapturedStep(lambda x, y: step_fn(x, y, cursor=cur), [ds.images, ds.labels],
                              warmup=2, bind_inputs=True)
        runner_k = None
        if kg > 1:
            def multi(x, y):
                for _ in range(kg):
                    out = step_fn(x, y, cursor=cur)
                return out

            runner_k = CapturedStep(multi, [ds.images, ds.labels], warmup=1, bind_inputs=True)
        with torch.no_grad():
            flat.data.copy_(saved[0])
            flat.mark_updated()
            if buf is not None:
                buf.copy_(saved[1])
        optimizer.step_count = saved[2]

        def run(n=1):
            (runner_k if n > 1 else runner)(ds.images, ds.labels)
            optimizer.step_count += n  # the replays' updates (host-side count only)
    else:
        def run(n=1):
            step_fn(ds.images, ds.labels, cursor=cur)
    stats = {"losses": [], "steps": 0, "samples": 0, "comm_time": 0.0}
    pending = []  # (epoch, iters, step, pinned copy, event) awaiting print
    host = [torch.zeros(1, pin_memory=True) for _ in range(4)]

    def flush(block):
        while pending and (block or pending[0][4].query()):
            ep, it, st, hb, ev = pending.pop(0)
            ev.synchronize()
            avg = float(hb[0]) / log_every
            stats["losses"].append(avg)
            if writer is not None:
                writer.add_scalar("Train Loss", avg, st)
            print_fn('Device: %d epoch: %d, iters: %5d, loss: %.3f' % (rank or 0, ep, it, avg))

    def log_point(epoch, it, step):
        nonlocal nlog
        flush(False)
        hb = host[nlog % len(host)]
        if len(pending) >= len(host) - 1:
            flush(True)
        hb.copy_(step_fn.loss_sum, non_blocking=True)
        step_fn.loss_sum.zero_()
        ev = torch.cuda.Event()
        ev.record()
        pending.append((epoch + 1, it, step, hb, ev))
        nlog += 1

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step = 0
    nlog = 0
    samples = 0
    done = False
    step_fn.loss_sum.zero_()  # once: the running sum carries across epochs (reference)
    for epoch in range(num_epochs):
        cur.refill(epoch)  # this epoch's shard order (set_epoch), cursor rewound
        i = 0  # batches done in this epoch
        while i < cur.nbatch:
            n = kg if (kg > 1 and i % kg == 0 and i + kg <= cur.nbatch
                       and (max_steps is None or step + kg <= max_steps)) else 1
            run(n)
            i += n
            step += n
            samples += n * loader.batch_size
            if i % log_every == 0:  # a k-step block never straddles a log point (k | log_every)
                log_point(epoch, i, step)
            if max_steps is not None and step >= max_steps:
                done = True
                break
        if not done and tail:
            # the shard's partial last batch: one eager fused step on the gathered rows
            xt = ds.images.index_select(0, cur.tail)
            yt = ds.labels.index_select(0, cur.tail)
            step_fn(xt, yt)
            i += 1
            step += 1
            samples += tail
            if i % log_every == 0:
                log_point(epoch, i, step)
            if max_steps is not None and step >= max_steps:
                done = True
        if done:
            break
    torch.cuda.synchronize()
    stats["train_time"] = time.perf_counter() - t0
    flush(True)
    stats["steps"] = step
    stats["samples"] = samples
    stats["graph_steps"] = kg if graph else None
    print_fn("Training Finished!")
    if writer is not None:
        writer.flush()
    return stats


@torch.no_grad()
def test(model, test_loader, print_fn=print):
    model.eval()
    size = len(test_loader.dataset)
    correct = None
    print_fn("testing ...")
    for inputs, labels in test_loader:
        out = model(inputs)
        correct = count_correct(out, labels, correct)
    c = int(correct) if correct is not None else 0
    print_fn('\nTest set: Accuracy: {}/{} ({:.2f}%)\n'.format(c, size, 100 * c / size))
    model.train()
    return c / max(size, 1)
