"""Fused flat optimiser kernels vs the reference formulas (fp32 PyTorch)."""
import math

import pytest
import torch

from dmlab.ops._native import lib

pytestmark = pytest.mark.gpu


def _ref_sgd(p, g, buf, lr, mom, damp, wd, nesterov, gscale, first):
    d = g * gscale + wd * p
    if mom != 0:
        buf = d.clone() if first else mom * buf + (1 - damp) * d
        d = d + mom * buf if nesterov else buf
    return p - lr * d, buf


@pytest.mark.parametrize("n", [1, 7, 4096, 51902, 1 << 20])
@pytest.mark.parametrize("mom,nesterov", [(0.0, False), (0.9, False), (0.9, True)])
def test_sgd_matches_reference(dev, n, mom, nesterov):
    torch.manual_seed(0)
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    buf = torch.zeros(n, device=dev)
    pr, br = p.clone(), buf.clone()
    pbf = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for step in range(3):
        first = step == 0
        pr, br = _ref_sgd(pr, g, br, 0.01, mom, 0.0, 1e-4, nesterov, 0.5, first)
        lib().sgd_step(p, g, buf, pbf, 0.01, mom, 0.0, 1e-4, 0.5, nesterov, first)
    torch.testing.assert_close(p, pr, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(pbf, p.bfloat16(), rtol=0, atol=0)
    if mom:
        torch.testing.assert_close(buf, br, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("bias_correction", [False, True])
def test_adam_matches_reference(dev, bias_correction):
    torch.manual_seed(1)
    n = 51902
    p = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    lr, b1, b2, eps = 5e-4 * math.sqrt(200), 0.9, 0.999, 1e-8
    for t in range(1, 4):
        g = torch.randn(n, device=dev)
        mr = b1 * mr + (1 - b1) * g
        vr = b2 * vr + (1 - b2) * g ** 2
        bc1 = 1 / (1 - b1 ** t) if bias_correction else 1.0
        bc2 = 1 / (1 - b2 ** t) if bias_correction else 1.0
        pr = pr - lr * (mr * bc1) / ((vr * bc2).sqrt() + eps)
        lib().adam_step(p, g, m, v, None, lr, b1, b2, eps, 0.0, 1.0, bc1, bc2)
    torch.testing.assert_close(p, pr, rtol=1e-5, atol=1e-5)


def test_cast_and_rows_mean(dev):
    x = torch.randn(3, 1001, device=dev)
    out = torch.empty(1001, device=dev)
    lib().rows_mean(x, out, 1 / 3)
    torch.testing.assert_close(out, x.mean(0), rtol=1e-6, atol=1e-6)
    xb = torch.empty(1001, device=dev, dtype=torch.bfloat16)
    lib().cast_f32_bf16(out, xb)
    torch.testing.assert_close(xb, out.bfloat16(), rtol=0, atol=0)
