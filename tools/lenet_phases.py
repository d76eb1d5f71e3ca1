"""Per-phase time of the fused LeNet sample kernel (csrc/lenet_fused.hip) from its probe.

The kernel stamps the 100 MHz real-time clock at its start and after every phase barrier when
``lenet_fused_step(..., probe=t)`` is given; this prints, per phase, the mean and max over the
batch's workgroups of the time since the previous stamp (10 ns resolution).

    python tools/lenet_phases.py [--batch 32] [--steps 50]
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

PHASES = ["stage input + weights", "conv1 + pool", "conv2 (channel halves) + combine + pool",
          "fc1", "fc2", "softmax CE", "fc2 dgrad", "fc1 dgrad", "records + unpool scatter",
          "conv2 dw + conv2 dgrad", "conv2 dgrad combine", "conv1 dw", "conv1 dw combine + bias"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    from dmlab.models import Net
    from dmlab.models.lenet_fused import FusedLeNetStep
    from dmlab.ops._native import lib
    from dmlab.optim import SGD

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = Net().to(dev)
    net._flatten()
    step = FusedLeNetStep(net, SGD(net.parameters(), lr=0.01, momentum=0.9))
    x = torch.rand(a.batch, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (a.batch,), device=dev)
    L = lib()
    nst = L.lenet_probe_stamps()
    probe = torch.zeros(a.batch * nst, dtype=torch.long, device=dev)
    rec, slab, rowloss = step._workspace(a.batch)
    flat = net.flat
    acc = None
    for s in range(a.steps):
        probe.zero_()
        L.lenet_fused_step(x, y, step.weights, rec, slab, rowloss, flat.grad, step.offsets, None,
                           None, 0.0, 0.0, 0.0, 0.0, 1.0, False, False, step.loss, probe=probe)
        torch.cuda.synchronize()
        t = probe.view(a.batch, nst).double()
        n = int((t[0] > 0).sum())
        d = (t[:, 1:n] - t[:, :n - 1]) * 10.0  # ns
        if s >= 5:
            acc = d if acc is None else acc + d
    acc = acc / (a.steps - 5) / 1e3  # us
    tot = acc.sum(1)
    print(f"fused LeNet sample kernel, batch {a.batch}: {tot.mean():.2f} us mean per workgroup "
          f"(start to last stamp), {a.steps - 5} steps")
    for i in range(acc.shape[1]):
        name = PHASES[i] if i < len(PHASES) else f"phase {i}"
        print(f"  {acc[:, i].mean():7.2f} us mean {acc[:, i].max():7.2f} max  {name}")


if __name__ == "__main__":
    main()
