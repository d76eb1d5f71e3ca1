"""hipGraph-captured training steps reproduce eager steps exactly."""
import copy

import pytest
import torch

from dmlab.models import Net, ResNet18
from dmlab.nn import cross_entropy
from dmlab.optim import SGD
from dmlab.utils.graph import CapturedStep

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["lenet", "resnet18"])
def test_captured_step_matches_eager(dev, kind):
    torch.manual_seed(0)
    if kind == "lenet":
        a = Net().to(dev)
        xs = [torch.rand(32, 1, 28, 28, device=dev) for _ in range(4)]
        ys = [torch.randint(0, 10, (32,), device=dev) for _ in range(4)]
    else:
        a = ResNet18(num_classes=10).to(dev)
        xs = [torch.rand(8, 3, 64, 64, device=dev) for _ in range(4)]
        ys = [torch.randint(0, 10, (8,), device=dev) for _ in range(4)]
    b = copy.deepcopy(a)
    b._flatten()
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9)

    def make_step(m, o):
        def step(x, y):
            loss = cross_entropy(m(x), y)
            o.zero_grad()
            loss.backward()
            o.step()
            return loss.detach()
        return step

    sa, sb = make_step(a, oa), make_step(b, ob)
    # eager reference: 3 warm-up steps on xs[0] (as CapturedStep does) then 4 steps
    for _ in range(3):
        sb(xs[0], ys[0])
    cap = CapturedStep(sa, [xs[0], ys[0]], warmup=3)
    for x, y in zip(xs, ys):
        la = cap(x, y).clone()
        lb = sb(x, y)
        torch.testing.assert_close(la, lb, rtol=1e-5, atol=1e-5)
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-4, atol=1e-5)
