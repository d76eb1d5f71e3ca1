"""NHWC bf16 ResNet kernels (implicit-GEMM conv fwd/dgrad/wgrad, BN, pooling) vs
PyTorch fp32 references computed on the same bf16-rounded inputs."""
import math

import pytest
import torch
import torch.nn.functional as F

from dmlab.ops._native import lib
from dmlab.ops.convbn import _cpad, pick_cfg

pytestmark = pytest.mark.gpu

GEOMS = [  # (N, H, Cin, Cout, k, stride, pad)
    (2, 8, 64, 64, 3, 1, 1),
    (2, 9, 64, 128, 3, 2, 1),
    (2, 8, 64, 128, 1, 2, 0),
    (3, 7, 256, 512, 3, 1, 1),
    (2, 14, 128, 256, 3, 2, 1),
    (2, 16, 3, 64, 7, 2, 3),  # stem (channels padded to 8)
]
# unit-stride shapes for the halo-staged kernel (cfg 39/41/42): wide rows (W=56: a
# 128-pixel block spans 4 rows), several 64-channel chunks, blocks crossing images
# (W=7), partial last block, 1x1 taps
HALO_GEOMS = [
    (3, 56, 64, 64, 3, 1, 1),
    (2, 28, 128, 128, 3, 1, 1),
    (5, 7, 128, 64, 3, 1, 1),
    (3, 14, 256, 256, 3, 1, 1),
    (2, 14, 64, 128, 1, 1, 0),
]
FWD_CFGS = list(range(9, 18)) + [39, 41, 42]
HALO_CFGS = [39, 41, 42]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


def _setup(dev, N, H, Cin, Cout, k, s, p, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(N, Cin, H, H, device=dev, generator=g).bfloat16()
    w = (torch.randn(Cout, Cin, k, k, device=dev, generator=g) / math.sqrt(Cin * k * k))
    cp = _cpad(Cin)
    xn = torch.empty(N, H, H, cp, device=dev, dtype=torch.bfloat16)
    lib().pack_input(x, xn)
    wf = torch.empty(Cout, k, k, cp, device=dev, dtype=torch.bfloat16)
    wd = torch.empty(Cin, k, k, Cout, device=dev, dtype=torch.bfloat16)
    lib().pack_weights(w.contiguous(), wf, wd, cp)
    return x, w, xn, wf, wd


@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("cfg", FWD_CFGS)
def test_conv_fwd_and_stats(dev, geom, cfg):
    _check_fwd(dev, geom, cfg)


@pytest.mark.parametrize("geom", HALO_GEOMS)
@pytest.mark.parametrize("cfg", [12] + HALO_CFGS)
def test_conv_fwd_halo(dev, geom, cfg):
    _check_fwd(dev, geom, cfg)


def _check_fwd(dev, geom, cfg):
    N, H, Cin, Cout, k, s, p = geom
    if cfg in (9, 12, 15) and Cout % 128:
        pytest.skip("128-wide tile needs Cout % 128 == 0")
    x, w, xn, wf, _ = _setup(dev, N, H, Cin, Cout, k, s, p)
    ref = F.conv2d(x.float(), w.bfloat16().float(), None, s, p)
    OH = ref.shape[2]
    y = torch.empty(N, OH, OH, Cout, device=dev, dtype=torch.bfloat16)
    M = N * OH * OH
    T = lib().conv_stats_rows(M, cfg, Cout)
    stats = torch.empty(T * 2 * Cout, device=dev)
    lib().conv_fwd(xn, wf, y, stats, None, k, k, s, p, cfg)
    assert _rel(_nchw(y), ref) < 6e-3
    st = stats.view(T, 2, Cout).sum(0)
    torch.testing.assert_close(st[0], ref.sum((0, 2, 3)), rtol=1e-3, atol=1e-2 * math.sqrt(M))
    torch.testing.assert_close(st[1], (ref * ref).sum((0, 2, 3)), rtol=1e-3, atol=1e-2 * math.sqrt(M))


def test_conv_fwd_add(dev):
    N, H, Cin, Cout, k, s, p = GEOMS[0]
    x, w, xn, wf, _ = _setup(dev, N, H, Cin, Cout, k, s, p)
    ref = F.conv2d(x.float(), w.bfloat16().float(), None, s, p)
    add = torch.randn(N, H, H, Cout, device=dev).bfloat16()
    y = torch.empty_like(add)
    lib().conv_fwd(xn, wf, y, None, add, k, k, s, p, pick_cfg(N * H * H, Cout))
    assert _rel(_nchw(y), ref + _nchw(add).float()) < 6e-3


@pytest.mark.parametrize("geom", GEOMS[:5])
@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("variant", [3, 4, 5])
def test_conv_dgrad(dev, geom, accumulate, variant):
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p)
    wb = w.bfloat16().float()
    OH = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, Cout, OH, OH, device=dev).bfloat16()
    ref = torch.nn.grad.conv2d_input((N, Cin, H, H), wb, dy.float(), s, p)
    dx = torch.randn(N, H, H, Cin, device=dev).bfloat16()
    base = dx.clone()
    lib().conv_dgrad(_nhwc(dy), wd, dx, k, k, s, p, dx if accumulate else None,
                     pick_cfg(N * H * H, Cin) % 3 + 3 * variant)
    if accumulate:
        ref = ref + _nchw(base).float()
    assert _rel(_nchw(dx), ref) < 6e-3


@pytest.mark.parametrize("geom", HALO_GEOMS + GEOMS[:2] + GEOMS[3:5])
@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("cfg", HALO_CFGS)
def test_conv_dgrad_halo(dev, geom, accumulate, cfg):
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p)
    wb = w.bfloat16().float()
    OH = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, Cout, OH, OH, device=dev).bfloat16()
    ref = torch.nn.grad.conv2d_input((N, Cin, H, H), wb, dy.float(), s, p)
    dx = torch.randn(N, H, H, Cin, device=dev).bfloat16()
    base = dx.clone()
    lib().conv_dgrad(_nhwc(dy), wd, dx, k, k, s, p, dx if accumulate else None, cfg)
    if accumulate:
        ref = ref + _nchw(base).float()
    assert _rel(_nchw(dx), ref) < 6e-3


@pytest.mark.parametrize("geom", GEOMS)
def test_conv_wgrad(dev, geom):
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p)
    OH = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, Cout, OH, OH, device=dev).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), s, p)
    M = N * OH * OH
    for beta in (0.0, 1.0):
        dw = torch.randn_like(w) if beta else torch.empty_like(w)
        base = dw.clone()
        big = 2 if Cout % 128 == 0 else 3
        for S, cfg in ((1, big), (3, 3), (2, 6)):
            K = k * k * _cpad(Cin)
            slab = torch.empty(S * Cout * K, device=dev)
            d = dw.clone()
            lib().conv_wgrad(xn, _nhwc(dy), d, slab, Cin, k, k, s, p, beta, S, cfg, False)
            exp = ref + (base if beta else 0)
            assert _rel(d, exp) < 2e-3, (S, cfg, beta)
    assert M > 0


@pytest.mark.parametrize("geom", [g for g in HALO_GEOMS if g[4] == 3] + [(2, 20, 64, 128, 3, 1, 1)])
@pytest.mark.parametrize("cfg", [4, 5])
@pytest.mark.parametrize("S", [1, 3, 7])
def test_conv_wgrad_halo(dev, geom, cfg, S):
    """Halo-staged 3x3 weight gradients: cfg 4 / 5 (9 / 3 taps per block); split-m slabs
    with slices ending mid-step, images crossing slices, several co tiles and ci chunks."""
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p)
    dy = torch.randn(N, Cout, H, H, device=dev).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), s, p)
    K = k * k * Cin
    slab = torch.empty(S * Cout * K, device=dev)
    d = torch.empty_like(w)
    lib().conv_wgrad(xn, _nhwc(dy), d, slab, Cin, k, k, s, p, 0.0, S, cfg, False)
    assert _rel(d, ref) < 2e-3


@pytest.mark.parametrize("C,M", [(64, 4096), (512, 98), (128, 1000)])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_forward_backward(dev, C, M, relu, res):
    torch.manual_seed(0)
    y = (torch.randn(M, C, device=dev) * 2 + 0.5).bfloat16()
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    r = torch.randn(M, C, device=dev).bfloat16() if res else None
    # reference
    yr = y.float().requires_grad_(True)
    g_ = gamma.clone().requires_grad_(True)
    b_ = beta.clone().requires_grad_(True)
    rm_ref, rv_ref = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    z = F.batch_norm(yr.t().unsqueeze(0), rm_ref, rv_ref, g_, b_, True, 0.1, 1e-5).squeeze(0).t()
    if res:
        z = z + r.float()
    out_ref = F.relu(z) if relu else z
    dout = torch.randn(M, C, device=dev).bfloat16()
    out_ref.backward(dout.float())
    # native: stats from a [T][2][C] slab (T=1)
    stats = torch.stack([y.float().sum(0), (y.float() ** 2).sum(0)]).reshape(-1).contiguous()
    f = dict(device=dev, dtype=torch.float32)
    scale, shift, mean, invstd = (torch.empty(C, **f) for _ in range(4))
    rm, rv = torch.zeros(C, **f), torch.ones(C, **f)
    lib().bn_stats_finalize(stats, 1, float(M), gamma, beta, rm, rv, 0.1, 1e-5, scale, shift, mean,
                            invstd, torch.empty(512 * C, **f))
    torch.testing.assert_close(rm, rm_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rv, rv_ref, rtol=1e-3, atol=1e-3)
    y4, out = y.view(1, 1, M, C), torch.empty(1, 1, M, C, device=dev, dtype=torch.bfloat16)
    lib().bn_apply(y4, r.view(1, 1, M, C) if res else None, scale, shift, out, relu)
    assert _rel(out.view(M, C), out_ref.detach()) < 5e-3
    mask = None
    if relu:
        # 1-bit ReLU mask (bit j of byte i = out[chunk i, channel j] > 0), same out
        mask = torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
        out2 = torch.empty_like(out)
        lib().bn_apply(y4, r.view(1, 1, M, C) if res else None, scale, shift, out2, relu, mask=mask)
        assert torch.equal(out2, out)
        bits = (mask[:, None].int() >> torch.arange(8, device=dev)) & 1
        assert torch.equal(bits.view(M, C).bool(), out.view(M, C).float() > 0)
    modes = [0] if not relu else ([1, 4] if res else [1, 2, 4])  # 2: mask from y; 4: bits
    got = {}
    for mode in modes:
        dy = torch.empty_like(out)
        dres = torch.empty_like(out) if res else None
        dg, db = torch.zeros(C, **f), torch.zeros(C, **f)
        work = torch.empty(lib().bn_bwd_work(M, C), **f)
        lib().bn_backward(dout.view(1, 1, M, C), out, y4, mean, invstd, gamma, dg, db, 0.0, mode,
                          scale, shift, None, None, 3, 2, 1, dy, dres, work, mask=mask)
        assert _rel(dy.view(M, C), yr.grad) < 1e-2, mode
        assert _rel(dg, g_.grad) < 1e-2, mode
        assert _rel(db, b_.grad) < 1e-2, mode
        got[mode] = (dy, dg, db, dres)
    if 4 in got:  # the bit mask selects exactly the elements `out > 0` selects
        for a_, b_t in zip(got[4], got[1]):
            if a_ is not None:
                assert torch.equal(a_, b_t)


def test_maxpool_avgpool(dev):
    x = torch.randn(2, 64, 17, 17, device=dev).bfloat16()
    xn = _nhwc(x)
    y = torch.empty(2, 9, 9, 64, device=dev, dtype=torch.bfloat16)
    idx = torch.empty(2, 9, 9, 64, device=dev, dtype=torch.uint8)
    lib().maxpool_fwd(xn, y, idx, 3, 2, 1)
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    torch.testing.assert_close(_nchw(y).float(), yr, rtol=0, atol=0)
    dy = torch.randn_like(yr).bfloat16()
    yr.backward(dy.float())
    dx = torch.empty_like(xn)
    lib().maxpool_bwd(_nhwc(dy), idx, dx, 3, 2, 1)
    assert _rel(_nchw(dx), xr.grad) < 5e-3
    a = torch.empty(2, 64, device=dev, dtype=torch.bfloat16)
    lib().avgpool_fwd(xn, a)
    assert _rel(a, x.float().mean((2, 3))) < 5e-3
    g = torch.randn(2, 64, device=dev).bfloat16()
    dxa = torch.empty_like(xn)
    lib().avgpool_bwd(g, dxa)
    ref = (g.float() / (17 * 17))[:, None, None, :].expand(2, 17, 17, 64)
    assert _rel(dxa, ref) < 5e-3


@pytest.mark.parametrize("N,H", [(2, 32), (2, 224), (2, 18), (12, 224)])
@pytest.mark.parametrize("fcfg", [16, 60])
def test_stem_space_to_depth(dev, N, H, fcfg):
    """7x7/s2/p3 stem == 4x4/s1 conv over the space-to-depth packed input (cfg 60: the
    resident-weight stem kernel, csrc/conv_stem.hip; H=18: a partial last block; N=12 at 224:
    588 tiles, more than the persistent grid, so workgroups loop over several tiles)."""
    C, Co = 3, 64
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(N, C, H, H, device=dev, generator=g).bfloat16()
    w = torch.randn(Co, C, 7, 7, device=dev, generator=g) / math.sqrt(C * 49)
    xs = torch.empty(N, H // 2, H // 2, 16, device=dev, dtype=torch.bfloat16)
    lib().pack_input_s2d(x, xs)
    wf = torch.empty(Co, 4, 4, 16, device=dev, dtype=torch.bfloat16)
    lib().pack_weights_s2d(w.contiguous(), wf)
    ref = F.conv2d(x.float(), w.bfloat16().float(), None, 2, 3)
    y = torch.empty(N, H // 2, H // 2, Co, device=dev, dtype=torch.bfloat16)
    M = N * (H // 2) ** 2
    T = lib().conv_stats_rows(M, fcfg, Co)
    stats = torch.empty(T * 2 * Co, device=dev)
    lib().conv_fwd(xs, wf, y, stats, None, 4, 4, 1, 2, fcfg)
    assert _rel(_nchw(y), ref) < 6e-3
    st = stats.view(T, 2, Co).sum(0)
    torch.testing.assert_close(st[0], ref.sum((0, 2, 3)), rtol=1e-3, atol=1e-2 * math.sqrt(M))
    torch.testing.assert_close(st[1], (ref * ref).sum((0, 2, 3)), rtol=1e-3, atol=1e-2 * math.sqrt(M))
    dy = torch.randn_like(ref).bfloat16()
    dref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), 2, 3)
    for S, cfg in ((1, 3), (4, 3)):
        slab = torch.empty(S * Co * 256, device=dev)
        dw = torch.empty_like(w)
        lib().conv_wgrad(xs, _nhwc(dy), dw, slab, C, 4, 4, 1, 2, 0.0, S, cfg, True)
        assert _rel(dw, dref) < 2e-3


@pytest.mark.parametrize("layout", ["channels_last", "nchw"])
@pytest.mark.parametrize("H", [8, 224])
def test_stem_s2d_packing_layouts(dev, layout, H):
    """Space-to-depth packing of an fp32 image batch (channels_last takes the vectorised
    2-pixel kernel, NCHW the generic one): xs[n,i,j,(dy*2+dx)*3+c] = x[n,c,2i+dy,2j+dx]."""
    N, C = 3, 3
    x = torch.randn(N, C, H, H, device=dev)
    if layout == "channels_last":
        x = x.contiguous(memory_format=torch.channels_last)
    xs = torch.full((N, H // 2, H // 2, 16), 7.0, device=dev, dtype=torch.bfloat16)
    lib().pack_input_s2d(x, xs)
    ref = torch.zeros(N, H // 2, H // 2, 16, device=dev)
    for dy in range(2):
        for dx in range(2):
            sub = x[:, :, dy::2, dx::2].permute(0, 2, 3, 1)
            ref[..., (dy * 2 + dx) * 3:(dy * 2 + dx) * 3 + 3] = sub
    assert torch.equal(xs.float(), ref.bfloat16().float())


@pytest.mark.parametrize("layout", ["channels_last", "nchw_bf16"])
def test_stem_s2d_packing_gathers_rows(dev, layout):
    """The loader's gather fused into the packing: xs[n] = pack(x[idx[n]]) for a batch of
    row indices into a device-resident dataset (repeats allowed; out-of-range rows clamp)."""
    Nsrc, C, H = 11, 3, 32
    x = torch.randn(Nsrc, C, H, H, device=dev)
    if layout == "channels_last":
        x = x.contiguous(memory_format=torch.channels_last)
    else:
        x = x.bfloat16()
    idx = torch.tensor([7, 0, 10, 7, 3, 42], device=dev)
    xs = torch.empty(6, H // 2, H // 2, 16, device=dev, dtype=torch.bfloat16)
    lib().pack_input_s2d(x, xs, idx)
    ref = torch.empty_like(xs)
    lib().pack_input_s2d(x.index_select(0, idx.clamp(max=Nsrc - 1)).contiguous(
        memory_format=torch.channels_last if layout == "channels_last" else torch.contiguous_format),
        ref)
    assert torch.equal(xs, ref)


@pytest.mark.parametrize("H,W,C", [(18, 18, 64), (17, 17, 64), (56, 56, 32), (9, 14, 64)])
def test_bn_relu_maxpool_3x3s2_codes(dev, H, W, C):
    """The 3x3/s2 fused stem tail (two pooled outputs per thread) against torch: pooled
    values, argmax window codes (first max wins, 15 = window passes no gradient) and y at
    the argmax."""
    torch.manual_seed(1)
    N = 3
    y = (torch.randn(N, H, W, C, device=dev) * 1.5).bfloat16()
    scale = torch.rand(C, device=dev) + 0.5
    shift = torch.randn(C, device=dev) * 0.5
    z = (y.float() * scale + shift).relu().permute(0, 3, 1, 2)
    ref, ind = F.max_pool2d(z, 3, 2, 1, return_indices=True)
    OH, OW = ref.shape[2], ref.shape[3]
    out = torch.empty(N, OH, OW, C, device=dev, dtype=torch.bfloat16)
    idx = torch.empty(N, OH, OW, C, device=dev, dtype=torch.uint8)
    yarg = torch.empty_like(out)
    lib().bn_relu_maxpool(y, scale, shift, out, idx, 3, 2, 1, yarg=yarg)
    torch.testing.assert_close(_nchw(out).float(), ref.bfloat16().float(), rtol=0, atol=0)
    # torch's flat argmax -> (kh, kw) of the window at (2*oh - 1, 2*ow - 1)
    ih, iw = ind // W, ind % W
    oh = torch.arange(OH, device=dev).view(1, 1, OH, 1)
    ow = torch.arange(OW, device=dev).view(1, 1, 1, OW)
    code = (ih - (2 * oh - 1)) * 3 + (iw - (2 * ow - 1))
    code = torch.where(ref > 0, code, torch.full_like(code, 15))
    mism = (_nchw(idx).long() != code).float().mean().item()
    assert mism < 1e-3  # ties decided differently by fma rounding only
    yr = y.permute(0, 3, 1, 2).reshape(N, C, -1)
    yref = torch.gather(yr, 2, ind.reshape(N, C, -1)).view_as(ref)
    sel = (ref > 0) & (_nchw(idx).long() == code)
    assert torch.equal(_nchw(yarg)[sel], yref[sel])


@pytest.mark.parametrize("H,C", [(18, 64), (17, 64), (56, 32)])
def test_fused_bn_relu_maxpool_and_gather_backward(dev, H, C):
    """Stem tail: maxpool(relu(bn(y))) forward and the pool-gather BN backward (mode 3;
    even H takes the 2x2-quad gather kernels, odd H the per-pixel gather)."""
    torch.manual_seed(0)
    N = 2
    y = (torch.randn(N, H, H, C, device=dev) * 1.5).bfloat16()
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev) * 0.5
    yr = y.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    g_, b_ = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    z = F.batch_norm(yr, rm, rv, g_, b_, True, 0.1, 1e-5)
    pooled_ref = F.max_pool2d(F.relu(z), 3, 2, 1)
    dp = torch.randn_like(pooled_ref).bfloat16()
    pooled_ref.backward(dp.float())
    f = dict(device=dev, dtype=torch.float32)
    M = N * H * H
    yf = y.float().view(M, C)
    stats = torch.stack([yf.sum(0), (yf ** 2).sum(0)]).reshape(-1).contiguous()
    scale, shift, mean, invstd = (torch.empty(C, **f) for _ in range(4))
    lib().bn_stats_finalize(stats, 1, float(M), gamma, beta, None, None, 0.1, 1e-5, scale, shift,
                            mean, invstd, torch.empty(512 * C, **f))
    OH = (H + 2 - 3) // 2 + 1
    out = torch.empty(N, OH, OH, C, device=dev, dtype=torch.bfloat16)
    idx = torch.empty(N, OH, OH, C, device=dev, dtype=torch.uint8)
    lib().bn_relu_maxpool(y, scale, shift, out, idx, 3, 2, 1)
    assert _rel(_nchw(out), pooled_ref.detach()) < 5e-3
    dy = torch.empty_like(y)
    dg, db = torch.zeros(C, **f), torch.zeros(C, **f)
    work = torch.empty(lib().bn_bwd_work(M, C), **f)
    lib().bn_backward(None, None, y, mean, invstd, gamma, dg, db, 0.0, 3, scale, shift,
                      _nhwc(dp), idx, 3, 2, 1, dy, None, work)
    assert _rel(_nchw(dy), yr.grad) < 1e-2
    assert _rel(dg, g_.grad) < 1e-2
    assert _rel(db, b_.grad) < 1e-2
    # pooled-domain sums: y at the argmax (yarg) + the pooled grad give the same Σdz, Σdz·x̂
    yarg = torch.empty_like(out)
    out2 = torch.empty_like(out)
    lib().bn_relu_maxpool(y, scale, shift, out2, idx, 3, 2, 1, yarg=yarg)
    assert torch.equal(out2, out)
    part = torch.empty(lib().bn_bwd_rows(N * OH * OH, C) * 2 * C, **f)
    rows = lib().bn_bwd_reduce_masked(_nhwc(dp), yarg, mean, invstd, scale, shift, part)
    dy2 = torch.empty_like(y)
    dg2, db2 = torch.zeros(C, **f), torch.zeros(C, **f)
    lib().bn_backward(None, None, y, mean, invstd, gamma, dg2, db2, 0.0, 3, scale, shift,
                      _nhwc(dp), idx, 3, 2, 1, dy2, None, work, pre_slab=part, pre_rows=rows)
    assert _rel(dg2, g_.grad) < 1e-2
    assert _rel(db2, b_.grad) < 1e-2
    assert _rel(_nchw(dy2), yr.grad) < 1e-2
    torch.testing.assert_close(db2, db, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("T", [1, 100, 129, 6272])
@pytest.mark.parametrize("C", [64, 80, 512])
def test_bn_stats_finalize_slab_rows(dev, T, C):
    """Σ over a [T][2][C] per-tile statistics slab (direct and two-level reductions)."""
    M = 1000.0
    f = dict(device=dev, dtype=torch.float32)
    g = torch.Generator(device=dev).manual_seed(3)
    s = torch.rand(T, C, device=dev, generator=g) * 2.0
    q = s * s + torch.rand(T, C, device=dev, generator=g)
    stats = torch.stack([s, q], 1).contiguous()
    gamma, beta = torch.rand(C, **f) + 0.5, torch.randn(C, **f)
    scale, shift, mean, invstd = (torch.empty(C, **f) for _ in range(4))
    lib().bn_stats_finalize(stats.view(-1), T, M, gamma, beta, None, None, 0.1, 1e-5, scale, shift,
                            mean, invstd, torch.empty(512 * C, **f))
    sd, qd = s.double().sum(0), q.double().sum(0)
    mu = sd / M
    var = (qd / M - mu * mu).clamp_min(0)
    torch.testing.assert_close(mean.double(), mu, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(invstd.double(), 1 / torch.sqrt(var + 1e-5), rtol=1e-4, atol=1e-6)
    # num_batches_tracked is incremented once per call by the finalize kernel
    nb = torch.zeros(1, dtype=torch.int64, device=dev)
    for rep in range(2):
        out = [torch.empty(C, **f) for _ in range(4)]
        lib().bn_stats_finalize(stats.view(-1), T, M, gamma, beta, None, None, 0.1, 1e-5, *out,
                                torch.empty(512 * C, **f), nb)
        for a, b in zip(out, (scale, shift, mean, invstd)):
            assert torch.equal(a, b)
        assert int(nb.item()) == rep + 1


PREBN_GEOMS = [g for g in HALO_GEOMS if g[4] == 3] + [GEOMS[0], GEOMS[3], (4, 56, 64, 64, 3, 1, 1),
                                                         (2, 7, 512, 512, 3, 1, 1),
                                                         (2, 14, 64, 64, 3, 1, 1),
                                                         (5, 7, 64, 64, 3, 1, 1), (1, 9, 64, 64, 3, 1, 1)]


@pytest.mark.parametrize("geom", PREBN_GEOMS)
@pytest.mark.parametrize("cfg", HALO_CFGS + [90, 91, 92, 93])
def test_conv_fwd_prebn(dev, geom, cfg):
    """Halo conv consuming relu(y*scale + shift) of a RAW previous-conv output (fused
    BN-apply + ReLU in the staging); zero padding stays zero after the BN."""
    N, H, Cin, Cout, k, s, p = geom
    g = torch.Generator(device=dev).manual_seed(2)
    y = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
    sc = torch.rand(Cin, device=dev, generator=g) + 0.5
    sh = torch.randn(Cin, device=dev, generator=g) * 0.5
    w = torch.randn(Cout, Cin, k, k, device=dev, generator=g) / math.sqrt(Cin * k * k)
    wf = torch.empty(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16)
    lib().pack_weights(w.contiguous(), wf, None, Cin)
    a = (y.float() * sc + sh).relu().bfloat16().float()
    ref = F.conv2d(_nchw(a), w.bfloat16().float(), None, s, p)
    out = torch.empty(N, H, H, Cout, device=dev, dtype=torch.bfloat16)
    M = N * H * H
    T = lib().conv_stats_rows(M, cfg, Cout)
    stats = torch.empty(T * 2 * Cout, device=dev)
    lib().conv_fwd(y, wf, out, stats, None, k, k, s, p, cfg, pre_scale=sc, pre_shift=sh)
    assert _rel(_nchw(out), ref) < 6e-3
    st = stats.view(T, 2, Cout).sum(0)
    torch.testing.assert_close(st[0], ref.sum((0, 2, 3)), rtol=1e-3, atol=1e-2 * math.sqrt(M))


@pytest.mark.parametrize("geom", [g for g in HALO_GEOMS if g[4] == 3])
@pytest.mark.parametrize("cfg", [4, 5])
def test_conv_wgrad_prebn(dev, geom, cfg):
    N, H, Cin, Cout, k, s, p = geom
    g = torch.Generator(device=dev).manual_seed(3)
    y = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
    sc = torch.rand(Cin, device=dev, generator=g) + 0.5
    sh = torch.randn(Cin, device=dev, generator=g) * 0.5
    a = (y.float() * sc + sh).relu().bfloat16().float()
    dy = torch.randn(N, Cout, H, H, device=dev, generator=g).bfloat16()
    ref = torch.nn.grad.conv2d_weight(_nchw(a), (Cout, Cin, k, k), dy.float(), s, p)
    S = 2
    slab = torch.empty(S * Cout * k * k * Cin, device=dev)
    d = torch.empty(Cout, Cin, k, k, device=dev)
    lib().conv_wgrad(y, _nhwc(dy), d, slab, Cin, k, k, s, p, 0.0, S, cfg, False,
                     pre_scale=sc, pre_shift=sh)
    assert _rel(d, ref) < 2e-3


def test_pack_weights_tiled_matches_per_layer(dev):
    # one launch over several layers (3x3, 1x1, 7x7 stem with padded channels, Cout not a
    # multiple of 32 tiles' worth of ci) must be bit-identical to the per-layer packer
    shapes = [(64, 3, 7, 8), (64, 64, 3, 64), (128, 64, 1, 64), (96, 160, 3, 160), (512, 512, 3, 512)]
    g = torch.Generator(device=dev).manual_seed(3)
    rows, pre, outs = [], [0], []
    for co, ci, k, cp in shapes:
        w = torch.randn(co, ci, k, k, device=dev, generator=g)
        wf = torch.full((co, k, k, cp), 7.0, device=dev, dtype=torch.bfloat16)
        wd = torch.full((ci, k, k, co), 7.0, device=dev, dtype=torch.bfloat16)
        rf = torch.empty_like(wf)
        rd = torch.empty_like(wd)
        lib().pack_weights(w, rf, rd, cp)
        outs.append((w, wf, wd, rf, rd))
        rows.append([w.data_ptr(), wf.data_ptr(), wd.data_ptr(), co, ci, cp, k, k])
        pre.append(pre[-1] + -(-co // 32) * -(-max(cp, ci) // 32))
    desc = torch.tensor(rows, dtype=torch.int64).reshape(-1).to(dev)
    tpre = torch.tensor(pre, dtype=torch.int32).to(dev)
    lib().pack_weights_tiled(desc, tpre, pre[-1])
    torch.cuda.synchronize()
    for w, wf, wd, rf, rd in outs:
        assert torch.equal(wf, rf)
        assert torch.equal(wd, rd)


# pipelined LDS-DMA tiles (conv_pipe.hip, cfg 90/91/92): 3x3 and 1x1 taps, stride 1 and 2,
# odd and even K-step counts (1 step, 9 steps, 32 steps), several N tiles (XCD-grouped 1-D
# grid), partial last M tile, and channel counts the tile cannot take (falls back)
PIPE_GEOMS = [
    (3, 14, 256, 256, 3, 1, 1),
    (2, 14, 128, 256, 3, 2, 1),
    (2, 14, 256, 512, 1, 2, 0),
    (5, 7, 512, 512, 3, 1, 1),
    (2, 28, 128, 128, 3, 1, 1),
    (3, 56, 64, 64, 3, 1, 1),
    (2, 14, 2048, 256, 1, 1, 0),
    (2, 9, 64, 256, 1, 1, 0),
    (3, 20, 64, 128, 3, 1, 1),
]


@pytest.mark.parametrize("geom", PIPE_GEOMS)
@pytest.mark.parametrize("cfg", [90, 91, 92, 93])
def test_conv_fwd_pipe(dev, geom, cfg):
    _check_fwd(dev, geom, cfg)


@pytest.mark.parametrize("geom", PIPE_GEOMS[:6])
@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("cfg", [90, 91, 92, 93])
def test_conv_dgrad_pipe(dev, geom, accumulate, cfg):
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p)
    OH = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, Cout, OH, OH, device=dev).bfloat16()
    ref = torch.nn.grad.conv2d_input((N, Cin, H, H), w.bfloat16().float(), dy.float(), s, p)
    dx = torch.randn(N, H, H, Cin, device=dev).bfloat16()
    base = dx.clone()
    lib().conv_dgrad(_nhwc(dy), wd, dx, k, k, s, p, dx if accumulate else None, cfg)
    if accumulate:
        ref = ref + _nchw(base).float()
    assert _rel(_nchw(dx), ref) < 6e-3


# persistent resident-weight 64 -> 64 channel 3x3 conv (conv_res64.hip, cfg 80): the layer1
# shape, blocks crossing images (W = 7), a partial last tile (81 pixels), the widest supported
# row (W = 63: halo 256 rows), more tiles than workgroups (N = 16 at 56 x 56)
RES64_GEOMS = [(3, 56, 64, 64, 3, 1, 1), (2, 8, 64, 64, 3, 1, 1), (5, 7, 64, 64, 3, 1, 1),
               (1, 9, 64, 64, 3, 1, 1), (2, 63, 64, 64, 3, 1, 1), (16, 56, 64, 64, 3, 1, 1)]


@pytest.mark.parametrize("geom", RES64_GEOMS)
def test_conv_fwd_res64(dev, geom):
    _check_fwd(dev, geom, 80)


@pytest.mark.parametrize("geom", RES64_GEOMS[:4])
def test_conv_fwd_res64_add(dev, geom):
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, _ = _setup(dev, N, H, Cin, Cout, k, s, p, seed=5)
    ref = F.conv2d(x.float(), w.bfloat16().float(), None, s, p)
    add = torch.randn(N, H, H, Cout, device=dev).bfloat16()
    y = torch.empty_like(add)
    lib().conv_fwd(xn, wf, y, None, add, k, k, s, p, 80)
    assert _rel(_nchw(y), ref + _nchw(add).float()) < 6e-3


@pytest.mark.parametrize("geom", RES64_GEOMS)
def test_conv_fwd_prebn_res64(dev, geom):
    test_conv_fwd_prebn(dev, geom, 80)


@pytest.mark.parametrize("geom", RES64_GEOMS)
@pytest.mark.parametrize("accumulate", [False, True])
def test_conv_dgrad_res64(dev, geom, accumulate):
    test_conv_dgrad_halo(dev, geom, accumulate, 80)


def test_conv_res64_matches_halo_bitwise(dev):
    """Same fp32 accumulation order per output (taps outer, 16-deep k inner) as the halo tile:
    the persistent kernel's outputs equal cfg 39's bit for bit; the stats rows differ (one per
    workgroup) but sum to the same totals."""
    N, H, Cin, Cout, k, s, p = RES64_GEOMS[0]
    x, w, xn, wf, _ = _setup(dev, N, H, Cin, Cout, k, s, p, seed=7)
    outs = []
    for cfg in (39, 80):
        y = torch.empty(N, H, H, Cout, device=dev, dtype=torch.bfloat16)
        lib().conv_fwd(xn, wf, y, None, None, k, k, s, p, cfg)
        outs.append(y)
    assert torch.equal(outs[0], outs[1])


# row-streaming 64 -> 64 channel weight gradient (wgrad_res64.hip, wgrad cfg 8): one slab per
# workgroup, row ranges starting mid-image, several images per workgroup, W = 60 (widest)
WRES64_GEOMS = [(3, 56, 64, 64, 3, 1, 1), (2, 8, 64, 64, 3, 1, 1), (5, 7, 64, 64, 3, 1, 1),
                (1, 9, 64, 64, 3, 1, 1), (2, 60, 64, 64, 3, 1, 1)]


@pytest.mark.parametrize("geom", WRES64_GEOMS)
@pytest.mark.parametrize("S", [1, 5, "rows"])
@pytest.mark.parametrize("pre", [False, True])
def test_conv_wgrad_res64(dev, geom, S, pre):
    N, H, Cin, Cout, k, s, p = geom
    S = N * H if S == "rows" else min(S, N * H)
    g = torch.Generator(device=dev).manual_seed(11)
    y = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
    dy = torch.randn(N, Cout, H, H, device=dev, generator=g).bfloat16()
    kw = {}
    a = y.float()
    if pre:
        sc = torch.rand(Cin, device=dev, generator=g) + 0.5
        sh = torch.randn(Cin, device=dev, generator=g) * 0.5
        a = (y.float() * sc + sh).relu().bfloat16().float()
        kw = dict(pre_scale=sc, pre_shift=sh)
    ref = torch.nn.grad.conv2d_weight(_nchw(a), (Cout, Cin, k, k), dy.float(), s, p)
    slab = torch.full((S * Cout * k * k * Cin,), float("nan"), device=dev)
    d = torch.empty(Cout, Cin, k, k, device=dev)
    lib().conv_wgrad(y, _nhwc(dy), d, slab, Cin, k, k, s, p, 0.0, S, 8, False, **kw)
    assert _rel(d, ref) < 2e-3


def test_conv_wgrad_res64_accumulates(dev):
    """beta = 1 adds onto the existing gradient (the step's accumulate path)."""
    N, H, Cin, Cout, k, s, p = WRES64_GEOMS[1]
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p, seed=4)
    dy = torch.randn(N, Cout, H, H, device=dev).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), s, p)
    base = torch.randn_like(w)
    d = base.clone()
    slab = torch.empty(4 * Cout * k * k * Cin, device=dev)
    lib().conv_wgrad(xn, _nhwc(dy), d, slab, Cin, k, k, s, p, 1.0, 4, 8, False)
    assert _rel(d, ref + base) < 2e-3


@pytest.mark.parametrize("geom,cfg", [(RES64_GEOMS[0], 80), (RES64_GEOMS[2], 80),
                                      (HALO_GEOMS[1], 42), (HALO_GEOMS[2], 39),
                                      ((2, 14, 256, 256, 3, 1, 1), 90),
                                      ((3, 7, 512, 512, 3, 1, 1), 90),
                                      ((2, 8, 64, 64, 3, 1, 1), 13)])
def test_conv_dgrad_masked_add(dev, geom, cfg):
    """Fused identity skip: dx = dgrad(dy) + add * mask with the 1-bit mask (bit j of byte i =
    element 8i + j) applied in the epilogue equals the dgrad plus the materialised product,
    bit for bit."""
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p, seed=13)
    g = torch.Generator(device=dev).manual_seed(14)
    dy = torch.randn(N, Cout, H, H, device=dev, generator=g).bfloat16()
    add = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
    keep = torch.rand(N, H, H, Cin, device=dev, generator=g) > 0.4
    bits = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, device=dev, dtype=torch.uint8)
    mask = bits.sum(1, dtype=torch.uint8)
    dres = (add.float() * keep).bfloat16()
    ref = torch.empty(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    lib().conv_dgrad(_nhwc(dy), wd, ref, k, k, s, p, dres, cfg)
    out = torch.empty_like(ref)
    lib().conv_dgrad(_nhwc(dy), wd, out, k, k, s, p, add, cfg, add_mask=mask)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("geom", RES64_GEOMS)
def test_conv_dgrad_bn_reduce(dev, geom):
    """cfg 80 data gradient with the consumer BN's backward reduction in its epilogue: dx is
    bit-identical to the plain dgrad, and the per-workgroup rows add up to that BN's Σdz and
    Σdz·x̂ (dz = the stored bf16 dx where y*scale + shift > 0), against a float64 torch sum."""
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p, seed=21)
    g = torch.Generator(device=dev).manual_seed(22)
    dy = torch.randn(N, Cout, H, H, device=dev, generator=g).bfloat16()
    ref = torch.empty(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    lib().conv_dgrad(_nhwc(dy), wd, ref, k, k, s, p, None, 80)
    yb = (torch.randn(N, H, H, Cin, device=dev, generator=g) * 2 + 0.3).bfloat16()
    sc = torch.rand(Cin, device=dev, generator=g) + 0.5
    sh = torch.randn(Cin, device=dev, generator=g) * 0.5
    mu = torch.randn(Cin, device=dev, generator=g) * 0.2
    inv = torch.rand(Cin, device=dev, generator=g) + 0.5
    rows = lib().conv_stats_rows(N * H * H, 80, Cin)
    part = torch.full((rows * 2 * Cin,), float("nan"), device=dev)
    out = torch.empty_like(ref)
    lib().conv_dgrad(_nhwc(dy), wd, out, k, k, s, p, None, 80, red_y=yb, red_scale=sc,
                     red_shift=sh, red_mean=mu, red_invstd=inv, red_part=part)
    assert torch.equal(out, ref)
    yf = yb.double()
    dz = torch.where(yb.float() * sc + sh > 0, ref.double(), torch.zeros((), device=dev,
                                                                           dtype=torch.float64))
    want = torch.stack([dz.sum((0, 1, 2)), (dz * (yf - mu.double())).sum((0, 1, 2)) * inv.double()])
    got = part.view(rows, 2, Cin).double().sum(0)
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4 * float(want.abs().max()))


@pytest.mark.parametrize("geom,cfg", [(RES64_GEOMS[0], 80), (RES64_GEOMS[2], 80), (RES64_GEOMS[4], 80),
                                      ((2, 14, 256, 256, 3, 1, 1), 90), ((3, 7, 512, 512, 3, 1, 1), 90),
                                      ((2, 28, 128, 128, 3, 1, 1), 91), ((2, 28, 128, 128, 3, 1, 1), 92),
                                      ((2, 14, 64, 64, 3, 1, 1), 93),
                                      ((2, 28, 128, 128, 3, 1, 1), 42), ((3, 14, 256, 256, 3, 1, 1), 42)])
@pytest.mark.parametrize("masked", [False, True])
def test_conv_dgrad_bn_reduce_pipe(dev, geom, cfg, masked):
    """res64 (cfg 80), pipelined (cfg 90-93) or cfg 42 halo data gradient with the consumer
    BN's backward reduction in its epilogue: ReLU mask from y*scale + shift (a block's inner BN), or the residual block's
    1-bit mask together with the fused identity-skip add (the previous block's output BN).
    dx is bit-identical to the plain dgrad; the rows add up to Σdz, Σdz·x̂ (float64 torch)."""
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p, seed=31)
    g = torch.Generator(device=dev).manual_seed(32)
    dy = _nhwc(torch.randn(N, Cout, H, H, device=dev, generator=g).bfloat16())
    kw, keep_add = {}, None
    if masked:
        add = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
        keep_add = torch.rand(N, H, H, Cin, device=dev, generator=g) > 0.4
        kw = dict(add=add, add_mask=_bits(keep_add))
    ref = torch.empty(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    lib().conv_dgrad(dy, wd, ref, k, k, s, p, kw.get("add"), cfg, add_mask=kw.get("add_mask"))
    yb = (torch.randn(N, H, H, Cin, device=dev, generator=g) * 2 + 0.3).bfloat16()
    sc = torch.rand(Cin, device=dev, generator=g) + 0.5
    sh = torch.randn(Cin, device=dev, generator=g) * 0.5
    mu = torch.randn(Cin, device=dev, generator=g) * 0.2
    inv = torch.rand(Cin, device=dev, generator=g) + 0.5
    rows = lib().conv_stats_rows(N * H * H, cfg, Cin)
    part = torch.full((rows * 2 * Cin,), float("nan"), device=dev)
    out = torch.empty_like(ref)
    if masked:
        keep = torch.rand(N, H, H, Cin, device=dev, generator=g) > 0.5
        kw["red_mask"] = _bits(keep)
    else:
        keep = yb.float() * sc + sh > 0
    lib().conv_dgrad(dy, wd, out, k, k, s, p, kw.get("add"), cfg, add_mask=kw.get("add_mask"),
                     red_y=yb, red_scale=sc, red_shift=sh, red_mean=mu, red_invstd=inv,
                     red_part=part, red_mask=kw.get("red_mask"))
    assert torch.equal(out, ref)
    yf = yb.double()
    dz = torch.where(keep, ref.double(), torch.zeros((), device=dev, dtype=torch.float64))
    want = torch.stack([dz.sum((0, 1, 2)), (dz * (yf - mu.double())).sum((0, 1, 2)) * inv.double()])
    got = part.view(rows, 2, Cin).double().sum(0)
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4 * float(want.abs().max()))


def _bits(keep):
    """1-bit mask layout of the kernels: bit j of byte i = element 8i + j (NHWC order)."""
    b = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, device=keep.device, dtype=torch.uint8)
    return b.sum(1, dtype=torch.uint8)


# stride-2 3x3 weight gradient over the input parity planes (wgrad cfg 7): the first conv of
# layers 2-4, a small multi-image case (m-steps crossing images), partial last m-step
WS2_GEOMS = [(2, 56, 64, 128, 3, 2, 1), (3, 28, 128, 256, 3, 2, 1), (2, 14, 256, 512, 3, 2, 1),
             (5, 8, 64, 64, 3, 2, 1), (1, 6, 64, 64, 3, 2, 1)]


@pytest.mark.parametrize("geom", WS2_GEOMS)
@pytest.mark.parametrize("S", [1, 3, 16])
def test_conv_wgrad_s2(dev, geom, S):
    N, H, Cin, Cout, k, s, p = geom
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p, seed=7)
    OH = H // 2
    dy = torch.randn(N, Cout, OH, OH, device=dev).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), s, p)
    K = k * k * _cpad(Cin)
    S = max(1, min(S, N * OH * OH // 64))
    slab = torch.full((S * Cout * K,), float("nan"), device=dev)
    d = torch.empty_like(w)
    lib().conv_wgrad(xn, _nhwc(dy), d, slab, Cin, k, k, s, p, 0.0, S, 7, False)
    assert _rel(d, ref) < 2e-3
    base = torch.randn_like(w)
    d = base.clone()  # beta = 1: accumulate
    lib().conv_wgrad(xn, _nhwc(dy), d, slab, Cin, k, k, s, p, 1.0, S, 7, False)
    assert _rel(d, ref + base) < 2e-3


@pytest.mark.parametrize("S", [3, 11])
def test_wgrad_reduce_vector_matches_scalar(dev, S):
    """The slab reduce reads 16-byte vectors when the slab is 16-byte aligned and falls back
    to 4-byte loads otherwise (a slab view at a one-float offset): same summation order, so
    the two results are bit-identical (S = 11: split lanes and a predicated last batch)."""
    N, H, Cin, Cout, k, s, p = (4, 20, 64, 128, 3, 1, 1)
    x, w, xn, wf, wd = _setup(dev, N, H, Cin, Cout, k, s, p)
    dy = torch.randn(N, Cout, H, H, device=dev).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), s, p)
    n = S * Cout * k * k * Cin
    buf = torch.empty(n + 4, device=dev)
    out = []
    for off in (0, 1):
        d = torch.empty_like(w)
        lib().conv_wgrad(xn, _nhwc(dy), d, buf[off:off + n], Cin, k, k, s, p, 0.0, S, 4, False)
        out.append(d)
    assert torch.equal(out[0], out[1])
    assert _rel(out[0], ref) < 2e-3
