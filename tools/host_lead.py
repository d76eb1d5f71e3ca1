"""Is the ResNet-18 step host-bound?  Times how long the host takes to ENQUEUE K eager
steps (no sync inside the loop) against the wall time until the GPU has finished them.
If enqueue time per step is close to the total per step, the host (Python + launch
overhead) sets the pace, not the GPU.

    python tools/host_lead.py --steps 30 --warmup 5 [--batch 512]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=512)
    p.add_argument("--profile", default="", help="write a cProfile of the enqueue loop here")
    a = p.parse_args()
    from dmlab.models import ResNet18
    from dmlab.nn import cross_entropy
    from dmlab.optim import SGD
    from dmlab.parallel import DDP

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = ResNet18(num_classes=1000).to(dev)
    x = [torch.rand(a.batch, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
         for _ in range(2)]
    y = [torch.randint(0, 1000, (a.batch,), device=dev) for _ in range(2)]
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9)
    net = DDP(model)
    net.fold_average_into(opt)

    def step(i):
        loss = cross_entropy(net(x[i % 2]), y[i % 2])
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    prof = None
    if a.profile:
        import cProfile
        prof = cProfile.Profile()
    res = {}
    modes = ["plain", "autograd_1thread", "plain"] + (["profiled"] if prof else [])
    for n, mode in enumerate(modes):
        # backward on the calling thread, so cProfile also sees the native backward
        torch.autograd.set_multithreading_enabled(mode == "plain")
        for i in range(2):
            step(i)
        torch.cuda.synchronize()
        marks = []
        t0 = time.perf_counter()
        if mode == "profiled":
            prof.enable()
        for i in range(a.steps):
            step(i)
            marks.append(time.perf_counter())
        if mode == "profiled":
            prof.disable()
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        per = [(b - c) * 1e3 for b, c in zip(marks[1:], marks[:-1])]
        res[f"{n}_{mode}"] = {"enqueue_ms_per_step": round(t_enq / a.steps * 1e3, 3),
                     "total_ms_per_step": round(t_all / a.steps * 1e3, 3),
                     "host_step_ms_min": round(min(per), 3),
                     "host_step_ms_median": round(sorted(per)[len(per) // 2], 3)}
    print(json.dumps(res), flush=True)
    if prof:
        prof.dump_stats(a.profile)


if __name__ == "__main__":
    main()
