"""Measure stock PyTorch-ROCm (MIOpen/rocBLAS) on the reference workloads.

This is the comparison point named in BASELINE.md ("stock PyTorch-ROCm running
the same loop on the same box").  It prints one JSON line per configuration.
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from dmlab.models.reference import TorchLeNet, TorchResNet18  # noqa: E402


def bench(step, warmup, iters):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def run_resnet(batch, res, dtype, channels_last, warmup, iters):
    model = TorchResNet18().cuda()
    if channels_last:
        model = model.to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(batch, 3, res, res, device="cuda")
    if channels_last:
        x = x.to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
            loss = F.cross_entropy(model(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    t = bench(step, warmup, iters)
    return {"model": "resnet18", "batch": batch, "res": res, "dtype": str(dtype),
            "channels_last": channels_last, "ms_per_step": t * 1e3, "samples_per_s": batch / t}


def run_lenet(batch, warmup, iters, sync_every_step=True):
    model = TorchLeNet().cuda()
    opt = torch.optim.SGD(model.parameters(), lr=0.001, momentum=0.9)
    x = torch.rand(batch, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (batch,), device="cuda")

    def step():
        loss = F.cross_entropy(model(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        if sync_every_step:
            loss.item()  # reference syncs every iteration (task2/model.py:63)

    t = bench(step, warmup, iters)
    return {"model": "lenet", "batch": batch, "dtype": "fp32", "ms_per_step": t * 1e3,
            "samples_per_s": batch / t, "item_sync_per_step": sync_every_step}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--resnet-batches", default=None,
                    help="comma-separated ResNet-18 batches (channels_last bf16) only")
    ap.add_argument("--tuned", action="store_true",
                    help="torch.backends.cudnn.benchmark = True (MIOpen searches every conv "
                         "for its fastest solver on first use; longer warmup), ResNet in "
                         "both layouts, LeNet with and without the per-step loss.item()")
    a = ap.parse_args()
    print(json.dumps({"device": torch.cuda.get_device_name(0), "tuned": a.tuned}), flush=True)
    if a.tuned:
        torch.backends.cudnn.benchmark = True
        for b in (a.resnet_batches or "512").split(","):
            for cl in (True, False):
                r = run_resnet(int(b), 224, torch.bfloat16, cl, 15, 20)
                r["cudnn_benchmark"] = True
                print(json.dumps(r), flush=True)
        for sync in (True, False):
            r = run_lenet(32, 50, 500, sync_every_step=sync)
            r["cudnn_benchmark"] = True
            print(json.dumps(r), flush=True)
        return
    if a.resnet_batches:
        for b in a.resnet_batches.split(","):
            print(json.dumps(run_resnet(int(b), 224, torch.bfloat16, True, 5, 20)), flush=True)
        return
    for b in (32, 4096):
        print(json.dumps(run_lenet(b, 20, 100)), flush=True)
    for b, cl in ((256, True), (256, False), (128, True)):
        print(json.dumps(run_resnet(b, 224, torch.bfloat16, cl, 5, 20)), flush=True)


if __name__ == "__main__":
    main()
