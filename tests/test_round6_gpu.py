"""Round-6 GPU tests: the stride-2 data gradient with the block's 1x1/s2 projection merged in
as a second K segment of parity class (0,0), and that launch's BN-backward reduction epilogue
-- against fp32/float64 PyTorch (torch.nn.grad.conv2d_input of both convs)."""
import math

import pytest
import torch

from dmlab.ops._native import lib
from dmlab.ops.convbn import _cpad

pytestmark = pytest.mark.gpu

# (N, H, Cin, Cout): the projection blocks of ResNet-18 layers 2 / 3 / 4 at small batch, a
# multi-image small grid, a partial last row tile (N*H*H/4 not a multiple of 128)
S2_GEOMS = [(2, 56, 64, 128), (2, 28, 128, 256), (2, 14, 256, 512), (5, 8, 64, 64), (3, 10, 64, 128)]


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


def _bits(keep):
    b = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, device=keep.device, dtype=torch.uint8)
    return b.sum(1, dtype=torch.uint8)


def _pack(dev, w):
    cout, cin, k, _ = w.shape
    wf = torch.empty(cout, k, k, _cpad(cin), device=dev, dtype=torch.bfloat16)
    wd = torch.empty(cin, k, k, cout, device=dev, dtype=torch.bfloat16)
    lib().pack_weights(w.contiguous(), wf, wd, _cpad(cin))
    return wd


def _operands(dev, N, H, Cin, Cout, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    OH = H // 2
    w1 = torch.randn(Cout, Cin, 3, 3, device=dev, generator=g) / math.sqrt(9 * Cin)
    w2 = torch.randn(Cout, Cin, 1, 1, device=dev, generator=g) / math.sqrt(Cin)
    dy1 = torch.randn(N, Cout, OH, OH, device=dev, generator=g).bfloat16()
    dy2 = torch.randn(N, Cout, OH, OH, device=dev, generator=g).bfloat16()
    ref = (torch.nn.grad.conv2d_input((N, Cin, H, H), w1.bfloat16().double(), dy1.double(), 2, 1)
           + torch.nn.grad.conv2d_input((N, Cin, H, H), w2.bfloat16().double(), dy2.double(), 2, 0))
    return g, w1, w2, dy1, dy2, ref


def _cfg(Cin):
    return 15 if Cin % 128 == 0 else 13


@pytest.mark.parametrize("geom", S2_GEOMS)
@pytest.mark.parametrize("tile", ["auto", 12, 16, 11, 17, 90, 91, 92, 93])
def test_merged_shortcut_dgrad(dev, geom, tile):
    """dx = conv_T(dy1, W1; 3x3/s2/p1) + conv_T(dy2, W2; 1x1/s2/p0) in one launch vs float64."""
    N, H, Cin, Cout = geom
    cfg = _cfg(Cin) if tile == "auto" else tile
    if cfg in (12, 15) and Cin % 128:
        pytest.skip("128-wide tile needs Cin % 128 == 0")
    if cfg in (90, 91, 92, 93) and Cin % {90: 256, 91: 128, 92: 128, 93: 64}[cfg]:
        pytest.skip("pipelined tile needs Cin % its width == 0")
    _, w1, w2, dy1, dy2, ref = _operands(dev, N, H, Cin, Cout, 41)
    wd1, wd2 = _pack(dev, w1), _pack(dev, w2)
    dx = torch.full((N, H, H, Cin), float("nan"), device=dev, dtype=torch.bfloat16)
    lib().conv_dgrad(_nhwc(dy1), wd1, dx, 3, 3, 2, 1, None, cfg, dy2=_nhwc(dy2), wd2=wd2)
    err = ((_nchw(dx).double() - ref).norm() / ref.norm()).item()
    assert err < 4e-3, err
    # equals the two-launch path (3x3 dgrad, then the 1x1 accumulated in place) up to the one
    # bf16 rounding of the intermediate that the merge removes
    two = torch.empty_like(dx)
    lib().conv_dgrad(_nhwc(dy1), wd1, two, 3, 3, 2, 1, None, cfg)
    lib().conv_dgrad(_nhwc(dy2), wd2, two, 1, 1, 2, 0, two, cfg)
    err2 = ((_nchw(two).double() - ref).norm() / ref.norm()).item()
    assert err <= err2 * 1.05 + 1e-4, (err, err2)


@pytest.mark.parametrize("geom", S2_GEOMS[:4])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("tile", ["auto", 90, 93])
def test_merged_shortcut_dgrad_bn_reduce(dev, geom, masked, tile):
    """The merged launch also reduces the consumer BN's backward sums (Σdz, Σdz·x̂, dz = the
    stored bf16 dx under the ReLU mask y*sc + sh > 0 or the block's 1-bit mask): dx is
    bit-identical to the merged launch without the epilogue; the rows add up to float64."""
    N, H, Cin, Cout = geom
    cfg = _cfg(Cin) if tile == "auto" else tile
    if cfg in (90, 93) and Cin % {90: 256, 93: 64}[cfg]:
        pytest.skip("pipelined tile needs Cin % its width == 0")
    g, w1, w2, dy1, dy2, _ = _operands(dev, N, H, Cin, Cout, 43)
    wd1, wd2 = _pack(dev, w1), _pack(dev, w2)
    plain = torch.empty(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    lib().conv_dgrad(_nhwc(dy1), wd1, plain, 3, 3, 2, 1, None, cfg, dy2=_nhwc(dy2), wd2=wd2)
    yb = (torch.randn(N, H, H, Cin, device=dev, generator=g) * 2 + 0.3).bfloat16()
    sc = torch.rand(Cin, device=dev, generator=g) + 0.5
    sh = torch.randn(Cin, device=dev, generator=g) * 0.5
    mu = torch.randn(Cin, device=dev, generator=g) * 0.2
    inv = torch.rand(Cin, device=dev, generator=g) + 0.5
    rows = lib().dgrad_s2_red_rows(N, H, H, cfg)
    part = torch.full((rows * 2 * Cin,), float("nan"), device=dev)
    kw = {}
    if masked:
        keep = torch.rand(N, H, H, Cin, device=dev, generator=g) > 0.5
        kw["red_mask"] = _bits(keep)
    else:
        keep = yb.float() * sc + sh > 0
    out = torch.empty_like(plain)
    lib().conv_dgrad(_nhwc(dy1), wd1, out, 3, 3, 2, 1, None, cfg, red_y=yb, red_scale=sc,
                     red_shift=sh, red_mean=mu, red_invstd=inv, red_part=part,
                     dy2=_nhwc(dy2), wd2=wd2, **kw)
    assert torch.equal(out, plain)
    yf = yb.double()
    dz = torch.where(keep, plain.double(), torch.zeros((), device=dev, dtype=torch.float64))
    want = torch.stack([dz.sum((0, 1, 2)), (dz * (yf - mu.double())).sum((0, 1, 2)) * inv.double()])
    got = part.view(rows, 2, Cin).double().sum(0)
    assert torch.isfinite(got).all()
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4 * float(want.abs().max()))


def test_merged_shortcut_refuses_bad_operands(dev):
    N, H, Cin, Cout = S2_GEOMS[3]
    _, w1, w2, dy1, dy2, _ = _operands(dev, N, H, Cin, Cout, 44)
    wd1, wd2 = _pack(dev, w1), _pack(dev, w2)
    dx = torch.empty(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="dy2"):  # an accumulating launch cannot merge
        lib().conv_dgrad(_nhwc(dy1), wd1, dx, 3, 3, 2, 1, dx, 13, dy2=_nhwc(dy2), wd2=wd2)
    with pytest.raises(RuntimeError):  # pipelined tile that does not fit the geometry
        lib().conv_dgrad(_nhwc(dy1), wd1, dx, 3, 3, 2, 1, None, 90, dy2=_nhwc(dy2), wd2=wd2)
    N2, H2, Cin2, Cout2 = S2_GEOMS[1]
    _, v1, v2, e1, e2, _ = _operands(dev, N2, H2, Cin2, Cout2, 45)
    dx2 = torch.empty(N2, H2, H2, Cin2, device=dev, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="dy2"):  # pipelined: projection channels != dy's
        lib().conv_dgrad(_nhwc(e1), _pack(dev, v1), dx2, 3, 3, 2, 1, None, 91,
                         dy2=_nhwc(e2)[..., :64].contiguous(), wd2=_pack(dev, v2)[:, :, :, :64].contiguous())
    with pytest.raises(RuntimeError):  # wrong grid
        lib().conv_dgrad(_nhwc(dy1), wd1, dx, 3, 3, 2, 1, None, 13, dy2=_nhwc(dy2)[:, :-1],
                         wd2=wd2)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("merge", ["1", "0"])
def test_resnet18_step_merged_shortcut(dev, merge, monkeypatch):
    """A whole native ResNet-18 step with the merged projection data gradients (and their
    reduction epilogues) on and off: held to the error level of PyTorch's bf16 autocast against
    the fp32 step, per parameter (the criterion of test_resnet18_native_matches_reference), and
    the merged launches are really taken (layers 2-3 on igemm tiles; layer 4's pipelined tile
    keeps the separate launch)."""
    import copy

    import torch.nn.functional as F

    from dmlab.models import ResNet18
    from dmlab.nn import cross_entropy
    from dmlab.ops import _native

    monkeypatch.setenv("DMLAB_MERGE_SHORTCUT", merge)
    L = _native.lib()
    calls = []

    class Spy:
        def __getattr__(self, n):
            f = getattr(L, n)
            if n != "conv_dgrad":
                return f

            def wrapped(*a, **k):
                calls.append(("dy2" in k, "red_y" in k, a[5] if len(a) > 5 else k.get("stride")))
                return f(*a, **k)
            return wrapped

    spy = Spy()
    monkeypatch.setattr("dmlab.ops.convbn.lib", lambda: spy)
    torch.manual_seed(0)
    a = ResNet18(num_classes=10).to(dev)
    b = copy.deepcopy(a).set_backend("torch")
    b._flatten()
    c = copy.deepcopy(b)
    c._flatten()
    x = torch.rand(16, 3, 64, 64, device=dev)
    y = torch.randint(0, 10, (16,), device=dev)
    la = cross_entropy(a(x), y)
    lb = F.cross_entropy(b(x), y)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        oc = c(x)
    lc = F.cross_entropy(oc.float(), y)
    for l in (la, lb, lc):
        l.backward()
    assert abs(la.item() - lb.item()) < 5e-2 * max(1.0, abs(lb.item()))
    bad = []
    for (n, pa), (_, pb), (_, pc) in zip(a.named_parameters(), b.named_parameters(),
                                         c.named_parameters()):
        rn, rc = _rel(pa.grad, pb.grad), _rel(pc.grad, pb.grad)
        if rn > 1.5 * rc + 0.05:
            bad.append((n, rn, rc))
    assert not bad, bad
    merged = [c_ for c_ in calls if c_[0]]
    s2 = [c_ for c_ in calls if c_[2] == 2]
    if merge == "1":
        assert len(merged) >= 1 and all(m[1] for m in merged), calls
    else:
        assert not merged and s2, calls


# ------------------------------------------------------------------ BN-backward apply folded
# into the halo data gradient (cfg 42) and the 9-tap halo weight gradient (cfg 4)
FOLD_GEOMS = [(2, 28, 128, 128), (3, 14, 128, 128), (2, 8, 64, 128), (4, 7, 128, 64)]


def _fold_operands(dev, N, H, Cin, Cout, mode, seed):
    """dz (the BN's output gradient), y (its input), coef [3][Cout], scale/shift, mask, and the
    dy = a*dz' + b*y + c the kernels must stage, in float64 from the bf16 operands."""
    g = torch.Generator(device=dev).manual_seed(seed)
    dz = torch.randn(N, H, H, Cout, device=dev, generator=g).bfloat16()
    y = (torch.randn(N, H, H, Cout, device=dev, generator=g) * 1.5 + 0.2).bfloat16()
    coef = torch.randn(3, Cout, device=dev, generator=g) * torch.tensor([[1.0], [0.3], [0.1]], device=dev)
    sc = torch.rand(Cout, device=dev, generator=g) + 0.5
    sh = torch.randn(Cout, device=dev, generator=g) * 0.5
    keep = torch.rand(N, H, H, Cout, device=dev, generator=g) > 0.45
    kw = dict(bwd_y=y, bwd_coef=coef.reshape(-1).contiguous())
    if mode == 2:
        kw.update(bwd_scale=sc, bwd_shift=sh)
        pas = y.float() * sc + sh > 0
    elif mode == 4:
        kw["bwd_mask"] = _bits(keep)
        pas = keep
    else:
        pas = torch.ones_like(keep)
    d = torch.where(pas, dz.float(), torch.zeros((), device=dev))
    dy = coef[0] * d + coef[1] * y.float() + coef[2]
    return g, dz, y, kw, dy


@pytest.mark.parametrize("geom", FOLD_GEOMS)
@pytest.mark.parametrize("mode", [0, 2, 4])
def test_folded_bn_backward_dgrad(dev, geom, mode):
    """cfg 42 data gradient staging a*dz' + b*y + c itself == the same kernel on the
    materialised bf16 dy (bit-identical), and close to float64 conv2d_input of that dy."""
    N, H, Cin, Cout = geom
    g, dz, y, kw, dyf = _fold_operands(dev, N, H, Cin, Cout, mode, 51)
    w = torch.randn(Cout, Cin, 3, 3, device=dev, generator=g) / math.sqrt(9 * Cin)
    wd = _pack(dev, w)
    dyb = dyf.bfloat16()
    ref_kernel = torch.empty(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    lib().conv_dgrad(dyb, wd, ref_kernel, 3, 3, 1, 1, None, 42)
    out = torch.empty_like(ref_kernel)
    lib().conv_dgrad(dz, wd, out, 3, 3, 1, 1, None, 42, **kw)
    diff = (out.float() - ref_kernel.float()).abs().max().item()
    assert diff <= 2 ** -6 * ref_kernel.float().abs().max().item(), diff
    ref = torch.nn.grad.conv2d_input((N, Cin, H, H), w.bfloat16().double(),
                                     _nchw(dyb).double(), 1, 1)
    err = ((_nchw(out).double() - ref).norm() / ref.norm()).item()
    assert err < 6e-3, err


@pytest.mark.parametrize("geom", FOLD_GEOMS[:2])
@pytest.mark.parametrize("mode", [2, 4])
def test_folded_bn_backward_dgrad_with_reduce_and_skip(dev, geom, mode):
    """The folded operand together with the reduction epilogue and the masked skip add (the
    layer-2 c1 / c2 data gradients): dx and the part rows equal those of the unfolded launch
    on the materialised dy."""
    N, H, Cin, Cout = geom
    g, dz, y, kw, dyf = _fold_operands(dev, N, H, Cin, Cout, mode, 53)
    w = torch.randn(Cout, Cin, 3, 3, device=dev, generator=g) / math.sqrt(9 * Cin)
    wd = _pack(dev, w)
    add = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
    amask = _bits(torch.rand(N, H, H, Cin, device=dev, generator=g) > 0.5)
    yb = (torch.randn(N, H, H, Cin, device=dev, generator=g) * 2 + 0.3).bfloat16()
    rk = dict(red_y=yb, red_scale=torch.rand(Cin, device=dev, generator=g) + 0.5,
              red_shift=torch.randn(Cin, device=dev, generator=g) * 0.5,
              red_mean=torch.randn(Cin, device=dev, generator=g) * 0.2,
              red_invstd=torch.rand(Cin, device=dev, generator=g) + 0.5)
    rows = lib().conv_stats_rows(N * H * H, 42, Cin)
    outs = []
    for folded in (False, True):
        part = torch.full((rows * 2 * Cin,), float("nan"), device=dev)
        dx = torch.empty(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        src = dz if folded else dyf.bfloat16()
        lib().conv_dgrad(src, wd, dx, 3, 3, 1, 1, add, 42, add_mask=amask, red_part=part, **rk,
                         **(kw if folded else {}))
        outs.append((dx, part))
    (d0, p0), (d1, p1) = outs
    assert (d0.float() - d1.float()).abs().max().item() <= 2 ** -6 * d0.float().abs().max().item()
    torch.testing.assert_close(p1, p0, rtol=2e-3, atol=2e-3 * float(p0.abs().max()))


@pytest.mark.parametrize("geom", FOLD_GEOMS)
@pytest.mark.parametrize("mode", [0, 2, 4])
@pytest.mark.parametrize("pre", [False, True])
def test_folded_bn_backward_wgrad(dev, geom, mode, pre):
    """9-tap halo weight gradient staging a*dz' + b*y + c (with and without the fused pre-BN
    of its input) vs float64 conv2d_weight of the materialised dy."""
    N, H, Cin, Cout = geom
    g, dz, y, kw, dyf = _fold_operands(dev, N, H, Cin, Cout, mode, 55)
    x = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
    pk = {}
    xr = x.double()
    if pre:
        psc = torch.rand(Cin, device=dev, generator=g) + 0.5
        psh = torch.randn(Cin, device=dev, generator=g) * 0.5
        pk = dict(pre_scale=psc, pre_shift=psh)
        xr = torch.relu(x.float() * psc + psh).bfloat16().double()
    S = 4
    slab = torch.empty(S * Cout * 9 * Cin, device=dev)
    dw = torch.empty(Cout, Cin, 3, 3, device=dev)
    lib().conv_wgrad(x, dz, dw, slab, Cin, 3, 3, 1, 1, 0.0, S, 4, False, **pk, **kw)
    ref = torch.nn.grad.conv2d_weight(_nchw(xr), (Cout, Cin, 3, 3), _nchw(dyf.bfloat16()).double(), 1, 1)
    err = ((dw.double() - ref).norm() / ref.norm()).item()
    assert err < 2e-3, err


@pytest.mark.parametrize("fold", ["1", "0"])
def test_resnet18_step_bn_fold(dev, fold, monkeypatch):
    """Whole native ResNet-18 step with the layer-2 BN-backward applies folded (opt-in,
    DMLAB_BN_FOLD=1) and not: held to the bf16-autocast error envelope of the fp32 step per parameter, and the folded
    consumers are really used at 56x56 input scale (layer 2 at 28x28 halo tiles)."""
    import copy

    import torch.nn.functional as F

    from dmlab.models import ResNet18
    from dmlab.nn import cross_entropy
    from dmlab.ops import _native

    monkeypatch.setenv("DMLAB_BN_FOLD", fold)
    L = _native.lib()
    calls = []

    class Spy:
        def __getattr__(self, n):
            f = getattr(L, n)
            if n not in ("conv_dgrad", "conv_wgrad"):
                return f

            def wrapped(*a, **k):
                calls.append((n, "bwd_y" in k))
                return f(*a, **k)
            return wrapped

    spy = Spy()
    monkeypatch.setattr("dmlab.ops.convbn.lib", lambda: spy)
    torch.manual_seed(0)
    a = ResNet18(num_classes=10).to(dev)
    b = copy.deepcopy(a).set_backend("torch")
    b._flatten()
    c = copy.deepcopy(b)
    c._flatten()
    x = torch.rand(8, 3, 112, 112, device=dev)
    y = torch.randint(0, 10, (8,), device=dev)
    la = cross_entropy(a(x), y)
    lb = F.cross_entropy(b(x), y)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        oc = c(x)
    lc = F.cross_entropy(oc.float(), y)
    for l in (la, lb, lc):
        l.backward()
    assert abs(la.item() - lb.item()) < 5e-2 * max(1.0, abs(lb.item()))
    bad = []
    for (n, pa), (_, pb), (_, pc) in zip(a.named_parameters(), b.named_parameters(),
                                         c.named_parameters()):
        rn, rc = _rel(pa.grad, pb.grad), _rel(pc.grad, pb.grad)
        if rn > 1.5 * rc + 0.05:
            bad.append((n, rn, rc))
    assert not bad, bad
    folded = [c_ for c_ in calls if c_[1]]
    if fold == "1":
        assert len(folded) >= 2, calls  # dgrad + wgrad of at least one BN
    else:
        assert not folded, calls
