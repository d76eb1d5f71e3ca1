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

import time

import torch

from dmlab.nn.loss import count_correct


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
