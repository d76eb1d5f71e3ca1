"""Native path of :class:`dmlab.nn.layers.ConvBN` (NHWC bf16, ResNet family).

Forward : implicit-GEMM MFMA conv whose epilogue also emits per-tile Σy/Σy² →
          BN statistics finalize (+ running-stat update) → fused BN-apply
          [+ residual] [+ ReLU].
Backward: BN backward (reduce + apply, also emitting the residual-branch grad) →
          weight-gradient implicit GEMM (split-M fp32 slabs, fixed-order reduce into
          the OIHW fp32 grad slot) → data-gradient implicit GEMM (parity-class
          decomposition for stride 2), optionally fused with the skip-connection
          add.

Activations are plain contiguous ``[N, H, W, C]`` bf16 tensors.  Packed bf16
weights ([Cout][KH][KW][Cpad] for forward, [Cin][KH][KW][Cout] for dgrad) are
cached per layer and refreshed when the fp32 master changes.
"""
from __future__ import annotations

import contextlib
import math
import os

import torch

from ._native import lib


def _cpad(c):
    return max(8, (c + 7) // 8 * 8)


# forward-style kernel configs (csrc/conv_igemm.hip igemm_fwd): 9-17 v3 igemm tiles
# (tile = cfg % 3: 0 128x128, 1 128x64, 2 64x64; 12-13 32x32x16 MFMA, 15-17 two tiles of
# register prefetch); 20/21/39/41/42 halo-staged unit-stride tiles (csrc/conv_halo.hip);
# 60 the space-to-depth stem (csrc/conv_stem.hip); 90-93 pipelined LDS-DMA tiles
# (csrc/conv_pipe.hip).  Measured on MI355X (tools/bench_conv.py ->
# profiles/conv_kernels_r1.jsonl, conv_halo_tiles_b512_r1s4.jsonl):
#   * strided taps, stride-2 dgrad parity classes below 256 channels, 1x1/s2 below 256
#     channels: v3 tiles 15 / 13 / 11 by the block-count rule below (256-row tiles lose
#     there: one workgroup per CU exposes the staging latency).
TILE_CFG = (15, 13, 11)
_STEM_CFG = 60
# The round-3 A/B switches (DMLAB_NO_PIPE / NO_RES64 / NO_FUSED_SKIP / NO_DGRAD_RED /
# NO_WRES64 / WRES64_S / TAIL_WGRAD_FULL / WGRAD_BLOCKS / RES64_ADD_RED / STEM_CFG) are
# settled and removed; their measurements stay in docs/KERNELS.md and profiles/.


def dgrad_cfg(M, cin, k, stride, cout, H=0, W=0):
    """Kernel config of a data-gradient GEMM (dX has M pixels of ``cin`` channels)."""
    return pick_cfg(M, cin, k, stride, cout, W=W)


def pick_cfg(M, ncols, k=0, stride=0, cin=0, W=0):
    """Kernel config for a forward-style conv GEMM with M output pixels and ncols
    output channels.  ``k``/``stride``/``cin`` (kernel size, tap stride, input
    channels) enable the unit-stride halo kernel when they describe a k x k conv with
    unit tap stride over 64-channel-aligned input; ``W`` (image width, 0 = unknown)
    enables the resident-weight 64-channel kernel."""
    # 80: persistent resident-weight 64 -> 64 channel 3x3 conv (csrc/conv_res64.hip; its
    # 128-pixel tile's halo, 128 + 2W + 2 rows, must fit the 256-row LDS image; the input
    # below 1 GiB: its DMA pad pieces are addressed past 2^30)
    if (k == 3 and stride == 1 and cin == 64 and ncols == 64 and 0 < W <= 63
            and M * 128 < 2**30 - 2**14):
        return 80
    # 90: the pipelined LDS-DMA 256 x 256 tile (csrc/conv_pipe.hip), for >= 256 output
    # channels and 64-channel-aligned input, any tap geometry.  tools/bench_conv.py at batch
    # 1024 (profiles/conv_pipe_vs_halo_b1024_r3a.jsonl, TFLOP/s fwd/dgrad, best previous tile):
    #   layer3 3x3 975/1004 (41: 897/971), layer4 3x3 1151/1160 (41: 933/957),
    #   layer4 3x3/s2 1030/901 (15: 750/724), layer3 3x3/s2 fwd 778 (42: 690),
    #   layer4 1x1/s2 442/367 (15: 351/299); the 64/128-channel layers keep the halo tiles
    if ncols % 256 == 0 and cin % 64 == 0 and cin > 0:
        return 90
    if k == 3 and stride == 1 and cin % 64 == 0 and ncols % 64 == 0:
        # 64 output channels: the 256-pixel halo tile (2 x 2 waves of 128 x 32) amortises
        # the single-chunk halo prologue over twice the rows
        # 42: the 128-pixel BN-128 tile with two weight tiles of register prefetch;
        # 41: 256-pixel tile of 4 x 1 waves, each 64 x 64 (one LDS fragment read per MFMA
        # pair instead of 1.5; BN 64 doubles the column blocks).  tools/bench_conv.py
        # (profiles/conv_halo_tiles_b512_r1s4.jsonl, batch 512 / 256, TFLOP/s fwd/dgrad):
        #   layer2 (128 ch): 42 807/834, 20 761/818, 41 781/817   (b256: 42 647/681)
        #   layer3 (256 ch): 41 852/867, 42 834/840                (b256: 41 722/762)
        #   layer4 (512 ch): 41 856/867, 43 812/820                (b256: 41 822/848)
        #   layer1 (64 ch) : 39 612/683, 41 580/642
        if ncols >= 256:
            return 41
        return 42 if ncols >= 128 else 39
    if ncols % 128 == 0 and math.ceil(M / 128) * (ncols // 128) >= 192:
        t = 0  # 64x64 per wave beats the narrower tile even at ~1 block per CU
    elif math.ceil(M / 128) * math.ceil(ncols / 64) >= 480:
        t = 1
    else:
        t = 2
    return TILE_CFG[t]


# weight-gradient blocks per launch (m-split target): ~2 per CU.  These run on the side
# stream for the whole kernel and hold LDS the critical-path kernels need.  Measured
# (profiles/wgrad_blocks_r2c.jsonl, one call): 512 -> 44.2/44.4k img/s, 384 44.2k,
# 256 43.6/43.7k, 768 43.4k, 1024 43.4/43.5k; at 1024 images per GPU 512 -> 46.6k,
# 768 45.5-45.8k, 1024 46.0-46.2k (profiles/wgrad_blocks_b1024_r2c.jsonl); re-measured under
# the high-priority step stream in round 4: 160-1024 blocks and CU-masked weight-gradient
# streams all lose to 512 (profiles/wgrad_blocks_sidemask_ab_r4m.txt); round 6, a larger
# budget for layers 3-4 only (>= 256 output channels): 768 -1.5 %, 1024 -0.4 %
# (profiles/merged_shortcut_ab_r6.txt, "wide768" / "wide1024")
_WGRAD_BLOCKS = 512
_CUS = {}


def _cu_count():
    if not torch.cuda.is_available():
        return 256
    d = torch.cuda.current_device()
    if d not in _CUS:
        _CUS[d] = torch.cuda.get_device_properties(d).multi_processor_count
    return _CUS[d]


def _wgrad_plan(M, cout, K, k=0, stride=0, cin=0, force=None, W=0, rows=0, tail=False,
                even=0):
    """(cfg, S) for the weight-gradient GEMM dW[cout, K] = Σ_m dY[m, cout] X_col[m, K].

    cfg 8: row-streaming 64 -> 64 channel 3x3 kernel (csrc/wgrad_res64.hip; ``W`` = image
    width <= 60, ``rows`` = N*H image rows, S = 5/8 of the CUs); cfg 4/5: halo-staged 3x3
    unit-stride kernel (csrc/wgrad_halo.hip) with 9 / 3 taps per block; cfg 7: the stride-2
    3x3 kernel over the input's parity planes (same file); cfg 2/3/6: v2 igemm tiles
    128x128 / 64x128 / 64x256.
    S splits the m reduction over blocks into fp32 slabs summed by a fixed-order reduce:
    ~2 blocks per CU, each split >= 8 row steps, slab bytes S*cout*K*4."""
    halo = k == 3 and stride == 1 and cin % 64 == 0 and cout % 8 == 0
    res64 = k == 3 and stride == 1 and cin == 64 and cout == 64 and 0 < W <= 60 and rows > 0
    if force == 8 or (force is None and res64):
        # 5/8 of the CUs: the kernel runs on the side stream next to the dgrad + BN-backward
        # chain, and leaving that chain CUs of its own is 0.8% faster per step than one
        # workgroup on every CU (128-192 of 256 tie; profiles/wgrad_res64_slabs_ab_r3s3.txt)
        # ``tail``: the last conv before the stem, whose weight gradient runs next to the stem's
        # fused BN-backward + weight-gradient kernel at the end of the step, not next to a
        # dgrad chain: there it takes every CU (5/8 there, or the main stream instead of the
        # side stream, measure the same or slower: profiles/tail_wgrad_placement_ab_r4i.txt)
        S = _cu_count() if tail else max(1, _cu_count() * 5 // 8)
        return 8, max(1, min(rows, S))
    # ``even``: output width of a stride-2 conv whose output is exactly half the input in both
    # dims (0 otherwise); the 3x3 plane staging holds rows up to a width of 31
    # (1x1 projections on a one-tap variant of it measured slower than the igemm tile:
    # profiles/wgrad_s2_1x1_rejected_r4ao.txt)
    s2 = stride == 2 and k == 3 and cin % 64 == 0 and cout % 8 == 0 and 0 < even <= 31
    if force is not None:
        cfg = force
    elif s2:
        # stride-2 3x3 (first conv of layers 2-4): the parity-plane kernel, 9 taps per block
        cfg = 7
    elif halo:
        # 9 taps per block share every dY fragment, but a layer with few (cout, cin)
        # tiles then needs many m-splits (slab traffic ~ S * cout * K); 3 taps per block
        # triples the tiles
        cfg = 4 if math.ceil(cout / 64) * (cin // 64) >= 4 else 5
    else:
        cfg = 2 if cout % 128 == 0 else 3
    if cfg in (4, 5, 7):
        tiles = max(1, math.ceil(cout / 64) * (cin // 64) * (3 if cfg == 5 else 1))
        max_split = max(1, M // 512)
    else:
        bm = 128 if cfg == 2 else 64
        tiles = math.ceil(cout / bm) * math.ceil(K / (256 if cfg == 6 else 128))
        # >= 8 row steps of 64 per split: the small-K layers (1x1/s2 downsample: K = Cin)
        # have one or two output tiles, so the m-split is their only parallelism
        max_split = max(1, M // 512)
    # (2x / 4x more splits for cfg 7 measured -0.4 / -1.0 %: profiles/wgrad_s2_splits_ab_r4ap.txt)
    S = max(1, min(max_split, math.ceil(_WGRAD_BLOCKS / tiles)))
    return cfg, S


def as_nhwc(x, cpad=None):
    """Accept [N,H,W,C] bf16 (internal layout) or a user NCHW / channels_last tensor."""
    if x.dim() == 4 and x.dtype == torch.bfloat16 and x.is_contiguous() and getattr(x, "_dm_nhwc", False):
        return x
    N, C, H, W = x.shape
    cp = cpad or _cpad(C)
    y = torch.empty((N, H, W, cp), device=x.device, dtype=torch.bfloat16)
    lib().pack_input(x if x.dtype in (torch.float32, torch.bfloat16) else x.float(), y)
    return _mark(y)


def _mark(t):
    t._dm_nhwc = True
    return t


def empty_nhwc(N, H, W, C, like):
    return _mark(torch.empty((N, H, W, C), device=like.device, dtype=torch.bfloat16))


def use_s2d(layer, x):
    """7x7/s2 stem on a small-channel input with even H, W -> space-to-depth 4x4/s1."""
    return (layer.k == 7 and layer.stride == 2 and layer.padding == 3 and layer.cin <= 4
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0)


def packed_weights_s2d(layer):
    prog = layer._prog
    cache = getattr(layer, "_wcache_s2d", None)
    if cache is None or cache[0] != prog._wver:
        w = layer.weight.detach()
        wf = torch.empty((layer.cout, 4, 4, _cpad(4 * layer.cin)), device=w.device,
                         dtype=torch.bfloat16)
        lib().pack_weights_s2d(w, wf)
        cache = (prog._wver, wf)
        object.__setattr__(layer, "_wcache_s2d", cache)
    return cache[1]


def packed_weights_stem(layer):
    """[64][176] bf16 K-dense stem weights (k = ky*24 + kx*3 + c), cached per weight version."""
    prog = layer._prog
    cache = getattr(layer, "_wcache_k176", None)
    if cache is None or cache[0] != prog._wver:
        wk = cache[1] if cache is not None else torch.empty(
            (64, 176), device=layer.weight.device, dtype=torch.bfloat16)
        lib().stem_pack_weights(layer.weight.detach(), wk)
        cache = (prog._wver, wk)
        object.__setattr__(layer, "_wcache_k176", cache)
    return cache[1]


def _stem_image(x):
    """(images, idx) of a stem input: a loader batch by index (dmlab.data.Gathered) or an
    image tensor ((N,3,H,W) channels_last or (N,H,W,3)); None if it is neither."""
    if not isinstance(x, torch.Tensor):
        return x.images, x.idx
    if x.dim() == 4 and x.shape[1] == 3 and not getattr(x, "_dm_nhwc", False):
        if not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        return x, None
    return None


_STEM_FUSED_DEFAULT = "1"  # GPU-validated (tests/test_stem_fused.py); bench A/B +1.9 %


def stem_fused_ok(layer, x):
    """The K-dense fused stem (csrc/stem_fused.hip) serves this layer and input:
    7x7/s2/p3 conv 3 -> 64 + BN + ReLU + 3x3/s2/p1 max-pool, on a raw fp32 / bf16 / u8 image
    batch whose size the kernel supports, BN in training mode or eval (not eval-BN with
    gradients).  DMLAB_STEM_FUSED=0 selects the space-to-depth path (A/B)."""
    if os.environ.get("DMLAB_STEM_FUSED", _STEM_FUSED_DEFAULT) == "0":
        return False
    if not (getattr(layer, "pool_k", 0) == 3 and layer.pool_s == 2 and layer.pool_p == 1
            and layer.k == 7 and layer.stride == 2 and layer.padding == 3 and layer.cin == 3
            and layer.cout == 64 and layer.relu):
        return False
    im = _stem_image(x)
    if im is None:
        return False
    img = im[0]
    if img.dtype not in (torch.float32, torch.bfloat16, torch.uint8) or not img.is_cuda:
        return False
    H, W = (img.shape[2], img.shape[3]) if img.shape[1] == 3 else (img.shape[1], img.shape[2])
    return bool(lib().stem_fused_supported(H, W))


def _stem_fused_fwd(layer, x, ctx, train):
    """Fused stem forward: pooled BN-input extremum + window codes + BN statistics in one
    kernel, then BN + ReLU on the pooled tensor.  The conv output is never written."""
    from dmlab.data import input_affine

    L = lib()
    img, idx = _stem_image(x)
    B = idx.numel() if idx is not None else img.shape[0]
    H, W = (img.shape[2], img.shape[3]) if img.shape[1] == 3 else (img.shape[1], img.shape[2])
    PH, PW = H // 4, W // 4
    dev = img.device
    nsc, nbi = input_affine(img.dtype)
    wk = packed_weights_stem(layer)
    pext = empty_nhwc(B, PH, PW, 64, img)
    code = torch.empty((B, PH, PW, 32), device=dev, dtype=torch.uint8)
    grid = L.stem_fused_grid(B)
    f32 = dict(device=dev, dtype=torch.float32)
    scale = torch.empty(64, **f32)
    shift = torch.empty(64, **f32)
    use_batch = layer.training
    stats = torch.empty(grid * 128, **f32) if use_batch else None
    L.stem_fwd_fused(img, idx, nsc, nbi, wk, layer.bn_weight.detach(), pext, code, stats, grid)
    M = B * (H // 2) * (W // 2)
    if use_batch:
        mean = torch.empty(64, **f32)
        invstd = torch.empty(64, **f32)
        work = torch.empty(256 * 2 * 64, **f32)
        L.bn_stats_finalize(stats, grid, float(M), layer.bn_weight.detach(),
                            layer.bn_bias.detach(), layer.running_mean, layer.running_var,
                            layer.momentum, layer.eps, scale, shift, mean, invstd, work,
                            layer.num_batches_tracked)
    else:
        L.bn_eval_coeffs(layer.bn_weight.detach(), layer.bn_bias.detach(), layer.running_mean,
                         layer.running_var, layer.eps, scale, shift)
        mean = invstd = None
    out = empty_nhwc(B, PH, PW, 64, img)
    code4 = torch.empty((B, PH, PW, 32), device=dev, dtype=torch.uint8) if train else None
    L.stem_pool_apply(pext, code if train else None, scale, shift, out, code4)
    if train:
        ctx.update(fused_stem=True, img=img, gidx=idx, nsc=nsc, nbi=nbi, wk=wk, yarg=pext,
                   idx=code4, mean=mean, invstd=invstd, scale=scale, shift=shift, has_res=False,
                   first=True, s2d=False, pre=None, y=pext, x=None, M=M)
    return out


def _stem_fused_bwd(layer, dout, ctx):
    """Fused stem backward: BN-backward coefficients from the pooled-domain sums, then the
    weight gradient of dy = a*dz + b*y + cc with y recomputed from the raw input (never
    stored), reduced in fixed order into the OIHW gradient."""
    L = lib()
    dout = dout.contiguous()
    pext, code = ctx["yarg"], ctx["idx"]
    acc = 1.0 if layer.accumulate else 0.0
    pre_sums = ctx.pop("pre_sums", None) or {}
    if not pre_sums:
        part = torch.empty(L.bn_bwd_rows(pext.numel() // 64, 64) * 2 * 64, device=dout.device,
                           dtype=torch.float32)
        rows = L.bn_bwd_reduce_masked(dout, pext, ctx["mean"], ctx["invstd"], ctx["scale"],
                                      ctx["shift"], part)
        pre_sums = dict(pre_slab=part, pre_rows=rows)
    B = dout.shape[0]
    grid = L.stem_fused_grid(B)
    f32 = dict(device=dout.device, dtype=torch.float32)
    work = torch.empty(L.bn_bwd_work(ctx["M"], 64), **f32)
    dslab = torch.empty(L.stem_bwd_slab_len(grid), **f32)
    L.stem_bwd_fused2(ctx["img"], ctx["gidx"], ctx["nsc"], ctx["nbi"], ctx["wk"], dout, code,
                      ctx["mean"], ctx["invstd"], layer.bn_weight.detach(),
                      layer.grad_slot("bn_weight"), layer.grad_slot("bn_bias"), acc,
                      pre_sums["pre_slab"], pre_sums["pre_rows"], layer.grad_slot("weight"), acc,
                      work, dslab, grid)
    return None


def packed_weights(layer, need_wd=True):
    prog = layer._prog
    ver = prog._wver
    cache = getattr(layer, "_wcache", None)
    cp = _cpad(layer.cin)
    if cache is None or cache[0] != ver or (need_wd and cache[2] is None):
        w = layer.weight.detach()
        k = layer.k
        wf = torch.empty((layer.cout, k, k, cp), device=w.device, dtype=torch.bfloat16)
        wd = (torch.empty((layer.cin, k, k, layer.cout), device=w.device, dtype=torch.bfloat16)
              if need_wd else None)
        lib().pack_weights(w, wf, wd, cp)
        cache = (ver, wf, wd)
        object.__setattr__(layer, "_wcache", cache)
    return cache[1], cache[2]


def pack_all(prog, layers):
    """Refresh the packed bf16 weights (wf [Cout][KH][KW][Cpad], wd [Cin][KH][KW][Cout]) of
    every conv in ``layers`` with ONE kernel launch; :func:`packed_weights` then hits the
    cache.  Buffers persist across steps (stable pointers, graph-capturable); the device
    descriptor table is rebuilt only when a weight's storage moves."""
    ver = prog._wver
    layers = [m for m in layers if m.k * m.k <= 64][:32]
    if not layers:
        return
    key = tuple(m.weight.data_ptr() for m in layers)
    st = getattr(prog, "_pack_state", None)
    if st is None or st["key"] != key:
        dev = layers[0].weight.device
        bufs, rows, pre, tpre = [], [], [0], [0]
        for m in layers:
            cp = _cpad(m.cin)
            wf = torch.empty((m.cout, m.k, m.k, cp), device=dev, dtype=torch.bfloat16)
            wd = torch.empty((m.cin, m.k, m.k, m.cout), device=dev, dtype=torch.bfloat16)
            bufs.append((wf, wd))
            rows.append([m.weight.data_ptr(), wf.data_ptr(), wd.data_ptr(), m.cout, m.cin, cp,
                         m.k, m.k])
            pre.append(pre[-1] + m.cout * m.k * m.k * cp)
            tpre.append(tpre[-1] + -(-m.cout // 32) * -(-max(cp, m.cin) // 32))
        st = dict(key=key, bufs=bufs, total=pre[-1], ntiles=tpre[-1],
                  tprefix=torch.tensor(tpre, dtype=torch.int32).to(dev),
                  desc=torch.tensor(rows, dtype=torch.int64).reshape(-1).to(dev),
                  prefix=torch.tensor(pre, dtype=torch.int64).to(dev))
        object.__setattr__(prog, "_pack_state", st)
    for m in layers:
        assert m.weight.is_contiguous()
    lib().pack_weights_tiled(st["desc"], st["tprefix"], st["ntiles"])
    for m, (wf, wd) in zip(layers, st["bufs"]):
        object.__setattr__(m, "_wcache", (ver, wf, wd))


def _materialise(x, pre):
    """relu(x*scale + shift) as a tensor (fallback when a consumer cannot fuse it)."""
    out = empty_nhwc(*x.shape, x)
    lib().bn_apply(x, None, pre[0], pre[1], out, True)
    return out


def convbn_fwd(layer, x, ctx, train, residual=None, raw=False, pre=None):
    L = lib()
    if (residual is None and not raw and pre is None and (layer.training or not train)
            and stem_fused_ok(layer, x)):
        return _stem_fused_fwd(layer, x, ctx, train)
    gidx = None
    if not isinstance(x, torch.Tensor):  # dmlab.data.Gathered: a loader batch by row index
        if use_s2d(layer, x.images) and x.images.dtype in (torch.float32, torch.bfloat16):
            x, gidx = x.images, x.idx  # the s2d packing below gathers the rows itself
        else:
            x = x.materialize()
    first = not (x.dim() == 4 and getattr(x, "_dm_nhwc", False))
    s2d = first and use_s2d(layer, x)
    if s2d:
        # stem as a 4x4/s1 conv over the space-to-depth input (pad 2 top/left, 1 bottom/right)
        Nn, Cc, Hh, Ww = x.shape
        if gidx is not None:
            Nn = gidx.numel()
        xs = empty_nhwc(Nn, Hh // 2, Ww // 2, _cpad(4 * Cc), x)
        L.pack_input_s2d(x if x.dtype in (torch.float32, torch.bfloat16) else x.float(), xs, gidx)
        x = xs
        k, s, p = 4, 1, 2
        OH, OW = Hh // 2, Ww // 2
        wf = packed_weights_s2d(layer)
    else:
        x = as_nhwc(x, _cpad(layer.cin)) if first else x
        k, s, p = layer.k, layer.stride, layer.padding
        wf = None
    N, H, W, C = x.shape
    if not s2d:
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    M = N * OH * OW
    cout = layer.cout
    if wf is None:
        wf, _ = packed_weights(layer, need_wd=train and not first)
    y = empty_nhwc(N, OH, OW, cout, x)
    # s2d stem: the resident-weight stem kernel (60, csrc/conv_stem.hip) stages the weights
    # and the input halo once per 256 pixels (the v3 128x64 tile, 16, re-stages one 4-tap
    # K-slice per step: 382 TFLOP/s at batch 512, profiles/conv_stem_s2d_r1s4.jsonl)
    cfg = _STEM_CFG if s2d else pick_cfg(M, cout, k, s, C, W=OW if (OH, OW) == (H, W) else 0)
    pre_kw = {}
    if pre is not None:
        # the halo tiles (layer 2) and the layer-1 kernel normalise y1 on the fly; for the
        # pipelined tiles of layers 3-4 (cfg 90-93) materialising relu(bn1(y1)) is 1.7 % faster
        # per step than the in-LDS transform that delayed every pipeline stage (and layer 2
        # measures the same either way, as does layer 1: profiles/pipe_pre_materialise_ab_r4q.txt,
        # profiles/layer12_pre_materialise_ab_r4u.txt)
        if cfg in (39, 41, 42, 80):
            pre_kw = dict(pre_scale=pre[0], pre_shift=pre[1])
        else:  # not a halo-kernel shape: materialise the previous BN output
            x = _materialise(x, pre)
            pre = None
    f32 = dict(device=x.device, dtype=torch.float32)
    scale = torch.empty(cout, **f32)
    shift = torch.empty(cout, **f32)
    use_batch = layer.training
    if use_batch:
        T = L.conv_stats_rows(M, cfg, cout)
        stats = torch.empty(T * 2 * cout, **f32)
        L.conv_fwd(x, wf, y, stats, None, k, k, s, p, cfg, **pre_kw)
        mean = torch.empty(cout, **f32)
        invstd = torch.empty(cout, **f32)
        work = torch.empty(256 * 2 * cout, **f32)
        L.bn_stats_finalize(stats, T, float(M), layer.bn_weight.detach(), layer.bn_bias.detach(),
                            layer.running_mean, layer.running_var, layer.momentum, layer.eps,
                            scale, shift, mean, invstd, work, layer.num_batches_tracked)
    else:
        L.conv_fwd(x, wf, y, None, None, k, k, s, p, cfg, **pre_kw)
        L.bn_eval_coeffs(layer.bn_weight.detach(), layer.bn_bias.detach(), layer.running_mean,
                         layer.running_var, layer.eps, scale, shift)
        mean = invstd = None
    if train:
        ctx.update(x=x, y=y, mean=mean, invstd=invstd, has_res=residual is not None,
                   first=first, s2d=s2d, scale=scale, shift=shift, pre=pre)
    if raw:
        ctx["scale"], ctx["shift"] = scale, shift
        return y
    pool = getattr(layer, "pool_k", 0)
    if pool:
        # fused BN + ReLU + max-pool: the BN output is never materialised
        pk, ps, pp = layer.pool_k, layer.pool_s, layer.pool_p
        PH, PW = (OH + 2 * pp - pk) // ps + 1, (OW + 2 * pp - pk) // ps + 1
        out = empty_nhwc(N, PH, PW, cout, x)
        idx = torch.empty((N, PH, PW, cout), device=x.device, dtype=torch.uint8)
        # training: also keep y at each window's argmax, so the backward reduces the BN
        # sums over the pooled grid (see bn_relu_maxpool_kernel)
        yarg = empty_nhwc(N, PH, PW, cout, x) if (train and use_batch) else None
        L.bn_relu_maxpool(y, scale, shift, out, idx, pk, ps, pp, yarg=yarg)
        if train:
            ctx["idx"] = idx
            ctx["yarg"] = yarg
        return out
    out = empty_nhwc(N, OH, OW, cout, x)
    # residual + ReLU in training: a 1-bit (out > 0) mask is the backward's ReLU mask source
    # (the residual is not kept; re-reading `out` would cost 16x the bytes)
    mask = (torch.empty(out.numel() // 8, device=x.device, dtype=torch.uint8)
            if (train and residual is not None and layer.relu) else None)
    if callable(residual):  # a shortcut computed on another stream: join it here
        residual = residual()
    L.bn_apply(y, residual, scale, shift, out, layer.relu, mask=mask)
    if train and residual is not None:
        ctx["out"] = out
        ctx["mask"] = mask
    return out


# the v3 igemm tiles whose multi-geometry launch (a stride-2 data gradient's 4 parity classes)
# takes the merged projection segment and the BN-backward reduction epilogue
_MULTI_IGEMM = (11, 12, 13, 14, 15, 16, 17)
# ... and the pipelined tiles (layer 4), whose merged segment needs the projection's channel
# count equal to dy's (true of every ResNet projection)
_MULTI_PIPE = (90, 91, 92, 93)
# the layer-2 BN-backward apply folded into its halo consumers (DMLAB_BN_FOLD=1/0)
_BN_FOLD_DEFAULT = "0"
# DMLAB_RES64_RED_ADD default: layer-1 identity-block dgrads reduce the previous block's BN
_RES64_RED_ADD_DEFAULT = "1"


def _dgrad_red(L, red_for, cfg, stride, dx, allow_res64_add=False, complete_s2=False):
    """conv_dgrad kwargs that reduce the consumer BN's backward sums in the dgrad epilogue
    (see convbn_bwd ``red_for``); {} when the kernel or the layer does not qualify.

    cfg 80 (layer1), the pipelined tiles (90-93, layers 3-4) and the cfg 42 halo tile
    (layer2) take a plain ReLU consumer (mask from y*scale + shift > 0), the residual
    block's 1-bit mask, and the fused identity-skip add (the consumer's output gradient is
    dgrad + skip).  The stem (BN + ReLU + max-pool) reduces over the pooled grid: y is its
    value at each window's argmax (ctx["yarg"]), as bn_bwd_reduce_masked does."""
    rl, rctx = red_for
    # stride 2: only a data gradient that writes dx complete in one launch (the projection's
    # 1x1/s2 segment merged in, ``complete_s2``) can reduce its consumer's sums
    s2_ok = stride == 2 and complete_s2 and (cfg in _MULTI_IGEMM or cfg in _MULTI_PIPE)
    kernel_ok = (stride == 1 and (cfg == 80 or 90 <= cfg <= 93 or cfg == 42)) or s2_ok
    pool = getattr(rl, "pool_k", 0)
    y = rctx.get("yarg") if pool else rctx.get("y")
    if (not kernel_ok or not rl.relu or y is None
            or rctx.get("mean") is None or rctx.get("pre_sums") is not None
            or tuple(y.shape) != tuple(dx.shape)):
        return {}
    mask = None
    if rctx.get("has_res"):
        mask = rctx.get("mask")
        if mask is None:
            return {}
    # layer1's identity-block dgrads (res64 with the fused skip add, reducing the previous
    # block's BN): round 3 measured them 0.3% slower per step (the add/mask epilogue cost the
    # kernel ~100 us, more than the contended pass it saved: profiles/
    # dgrad_bn_reduce_ab_r3s3.txt, red9); with the round-6 packed/bit-extract reduction they
    # gain +0.26 % (profiles/res64_red_add_ab_r6.txt), default on; DMLAB_RES64_RED_ADD=0 opts
    # out (``allow_res64_add``: tests).  The STEM's pooled-grid sums in the last layer-1 dgrad
    # pay too: +0.5 % (the separate pooled reduce ran next to the full-CU tail weight gradient
    # at ~2 TB/s; profiles/side_stream_sweep_r4f.txt)
    if (cfg == 80 and mask is not None and not pool and not allow_res64_add
            and os.environ.get("DMLAB_RES64_RED_ADD", _RES64_RED_ADD_DEFAULT) != "1"):
        return {}
    N, H, W, C = dx.shape
    rows = (L.dgrad_s2_red_rows(N, H, W, cfg) if stride == 2
            else L.conv_stats_rows(N * H * W, cfg, C))
    part = torch.empty(rows * 2 * C, device=dx.device, dtype=torch.float32)
    rctx["pre_sums"] = dict(pre_slab=part, pre_rows=rows)
    kw = dict(red_y=y, red_scale=rctx["scale"], red_shift=rctx["shift"],
              red_mean=rctx["mean"], red_invstd=rctx["invstd"], red_part=part)
    if mask is not None:
        kw["red_mask"] = mask
    return kw


def convbn_bwd(layer, dout, ctx, need_dx, dx_add=None, dx_into=None, fused_skip=False,
               red_for=None, phase=0, shortcut=None):
    """Returns dx (or (dx, dres) when the forward had a residual input).

    ``dx_add``  : tensor added to dx in the dgrad epilogue (identity skip gradient), or
                  ("masked", dout, mask): dout * mask added there (the fused skip below)
    ``dx_into`` : accumulate dx in place into this tensor (downsample branch)
    ``fused_skip``: with a residual input and the forward's 1-bit ReLU mask, the residual
                  gradient dres = dout * mask is NOT materialised; the returned dres is
                  ("masked", dout, mask) for the consumer's dgrad epilogue (saves writing
                  and re-reading one activation-sized tensor per identity block)
    ``red_for``  : (layer, ctx) of the ConvBN + ReLU whose output gradient dx is.  When the
                  dgrad kernel supports it (cfg 80), that BN's backward reduction (Σdz, Σdz·x̂)
                  runs in this dgrad's epilogue and is left in its ctx["pre_sums"], so its
                  own backward skips the pass that re-reads dx and y
    ``phase``    : 0 = the whole backward; 1 = only the BatchNorm backward (dy kept in ctx),
                  on the caller's current stream; 2 = the weight and data gradients from
                  phase 1's dy (the caller has made the current stream wait for phase 1)
    ``shortcut`` : {"join": fn} of the block's 1x1/s2 projection (a stride-2 3x3 conv only):
                  fn() orders the current stream after the projection's BatchNorm backward and
                  returns (its dy, its packed data-gradient weights); when the dgrad tile can
                  merge it, the projection's data gradient becomes a second K segment of parity
                  class (0,0) in THIS launch (dx written once, complete, so ``red_for`` applies
                  too) and shortcut["merged"] is set -- the caller then skips its dgrad"""
    if ctx.get("fused_stem"):
        return _stem_fused_bwd(layer, dout, ctx)
    L = lib()
    x, y = ctx["x"], ctx["y"]
    N, OH, OW, cout = y.shape
    M = N * OH * OW
    s2d = ctx.get("s2d", False)
    k, s, p = (4, 1, 2) if s2d else (layer.k, layer.stride, layer.padding)
    acc = 1.0 if layer.accumulate else 0.0
    # ("masked", dout, mask): the upstream gradient is dout * mask (a projection shortcut fed
    # the block's unmaterialised residual gradient); the BN backward's mode 4 applies exactly
    # that mask, so no ReLU of its own is involved
    in_mask = None
    if isinstance(dout, tuple):
        _, dout, in_mask = dout
        assert not layer.relu and not ctx["has_res"], "masked upstream gradient: linear BN only"
    dout = dout.contiguous()
    pool = getattr(layer, "pool_k", 0)
    if phase == 2:
        assert not pool, "phase 2: a plain ConvBN"
        work, pre_sums = None, {}
    else:
        work = torch.empty(L.bn_bwd_work(M, cout), device=y.device, dtype=torch.float32)
        pre_sums = ctx.pop("pre_sums", None) or {}
    if pool and ctx.get("yarg") is not None and not pre_sums:
        # stem: Σdz, Σdz·x̂ over the pooled grid (pooled grad masked at the argmax, x̂ from
        # y at the argmax) -- reads 2 pooled-size tensors instead of y + grad + codes
        Mp = ctx["yarg"].numel() // cout
        part = torch.empty(L.bn_bwd_rows(Mp, cout) * 2 * cout, device=y.device,
                           dtype=torch.float32)
        rows = L.bn_bwd_reduce_masked(dout, ctx["yarg"], ctx["mean"], ctx["invstd"], ctx["scale"],
                                      ctx["shift"], part)
        pre_sums = dict(pre_slab=part, pre_rows=rows)
    stem_ok = (pool and s2d and pre_sums and ctx["first"] and not ctx["has_res"]
               and L.stem_bwd_fused_supported(y, x))
    if stem_ok:
        # stem: BN-backward apply fused into the s2d weight gradient -- the full-resolution
        # dy is never written (csrc/conv_stem.hip stem_wgrad_ws_kernel)
        slab = torch.empty(L.stem_bwd_slab_floats(N, OH), device=y.device, dtype=torch.float32)
        L.stem_bwd_fused(y, ctx["mean"], ctx["invstd"], layer.bn_weight.detach(),
                         layer.grad_slot("bn_weight"), layer.grad_slot("bn_bias"), acc,
                         ctx["scale"], ctx["shift"], dout, ctx["idx"], pre_sums["pre_slab"],
                         pre_sums["pre_rows"], x, layer.cin, layer.grad_slot("weight"), acc,
                         work, slab)
        return None
    if pool:
        mode = 3       # dz gathered from the max-pool gradient, ReLU mask from y
    elif in_mask is not None:
        mode = 4       # dz = dout * the residual block's 1-bit mask
    elif not layer.relu:
        mode = 0
    elif ctx["has_res"]:
        # mask needs the residual: the forward's 1-bit mask (4), or the saved output (1)
        mode = 4 if ctx.get("mask") is not None else 1
    else:
        mode = 2       # mask recomputed from y (no `out` read)
    C = x.shape[3]
    K = k * k * C
    same = not s2d and (OH, OW) == tuple(x.shape[1:3])
    # red_for is the stem (a pooled ConvBN) only for the first block's c1: the step's last conv
    tail = red_for is not None and bool(getattr(red_for[0], "pool_k", 0))
    even = OW if (not s2d and 2 * OH == x.shape[1] and 2 * OW == x.shape[2]) else 0
    wcfg, S = _wgrad_plan(M, cout, K, k, s, C, W=OW if same else 0, rows=N * OH if same else 0,
                          tail=tail, even=even)
    masked_res = fused_skip and ctx["has_res"] and mode == 4
    # The BN-backward apply folded into both consumers (layer 2's halo data gradient, cfg 42,
    # and the 9-tap halo weight gradient, cfg 4): they stage dy = a*dz' + b*y + c themselves
    # from dout and y, so the apply pass and its dy tensor do not exist
    # (DMLAB_BN_FOLD=0: the separate apply pass)
    fold = False
    if (phase == 0 and not pool and mode in (0, 2, 4) and need_dx and not ctx["first"]
            and dx_into is None and not (ctx["has_res"] and not masked_res)
            and s == 1 and k == 3 and p == 1 and wcfg == 4
            and os.environ.get("DMLAB_BN_FOLD", _BN_FOLD_DEFAULT) != "0"):
        Nx, Hx, Wx, Cx = x.shape
        fold = (dgrad_cfg(Nx * Hx * Wx, Cx, k, s, cout, Hx, Wx) == 42
                and L.bn_fold_supported(Nx, Hx, Wx, Cx, cout))
    bwd_kw = {}
    if fold:
        L.bn_backward(dout, None, y, ctx["mean"], ctx["invstd"], layer.bn_weight.detach(),
                      layer.grad_slot("bn_weight"), layer.grad_slot("bn_bias"), acc, mode,
                      ctx["scale"], ctx["shift"], None, None, 3, 2, 1, None, None, work,
                      mask=in_mask if in_mask is not None else ctx.get("mask"), **pre_sums)
        off = L.bn_bwd_coef_offset(M, cout, bool(pre_sums))
        bwd_kw = dict(bwd_y=y, bwd_coef=work[off:off + 3 * cout])
        if mode == 2:
            bwd_kw.update(bwd_scale=ctx["scale"], bwd_shift=ctx["shift"])
        elif mode == 4:
            bwd_kw["bwd_mask"] = in_mask if in_mask is not None else ctx["mask"]
        dy, dres = dout, None  # the consumers' dY operand is the BN's output gradient
    elif phase == 2:
        dy, dres = ctx.pop("_bn_out")
        # allocated on the phase-1 stream, read here and on the weight-gradient stream
        dy.record_stream(torch.cuda.current_stream())
        if dres is not None:
            dres.record_stream(torch.cuda.current_stream())
    else:
        dy = empty_nhwc(N, OH, OW, cout, y)
        dres = empty_nhwc(N, OH, OW, cout, y) if (ctx["has_res"] and not masked_res) else None
        L.bn_backward(None if pool else dout, ctx.get("out"), y, ctx["mean"], ctx["invstd"],
                      layer.bn_weight.detach(), layer.grad_slot("bn_weight"),
                      layer.grad_slot("bn_bias"), acc, mode, ctx["scale"], ctx["shift"],
                      dout if pool else None, ctx.get("idx"),
                      getattr(layer, "pool_k", 3), getattr(layer, "pool_s", 2),
                      getattr(layer, "pool_p", 1), dy, dres, work,
                      mask=in_mask if in_mask is not None else ctx.get("mask"), **pre_sums)
        if phase == 1:
            ctx["_bn_out"] = (dy, dres)
            return None
    # weight gradient: on the Program's side stream when it has one (off the critical
    # path; overlaps the following dgrad / BN-backward chain).  Tensors it reads that the
    # main stream allocated are recorded on the side stream so the caching allocator does
    # not hand their memory out again before the wgrad has read them.
    pre = ctx.get("pre")
    side = getattr(layer._prog, "_wgrad_stream", None)

    def launch_wgrad():
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
            for t in (x, dy) + (tuple(pre) if pre is not None else ()) + tuple(bwd_kw.values()):
                t.record_stream(side)
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            slab = torch.empty(S * cout * K, device=y.device, dtype=torch.float32)
            pre_kw = {}
            xw = x
            if pre is not None:
                if wcfg in (4, 5, 8):
                    pre_kw = dict(pre_scale=pre[0], pre_shift=pre[1])
                else:
                    xw = _materialise(x, pre)
            L.conv_wgrad(xw, dy, layer.grad_slot("weight"), slab, layer.cin, k, k, s, p, acc, S,
                         wcfg, s2d, **pre_kw, **bwd_kw)

    launch_wgrad()
    dx = None
    if need_dx and not ctx["first"]:
        _, wd = packed_weights(layer, need_wd=True)
        N_, H, W, Cin = x.shape
        cfg = dgrad_cfg(N_ * H * W, Cin, k, s, cout, H, W)
        if dx_into is not None:
            dx = dx_into
            L.conv_dgrad(dy, wd, dx_into, k, k, s, p, dx_into, cfg)
        else:
            dx = empty_nhwc(N_, H, W, Cin, x)
            merge_kw = {}
            if (shortcut is not None and s == 2 and k == 3 and p == 1 and dx_add is None
                    and (cfg in _MULTI_IGEMM
                         or (cfg in _MULTI_PIPE and os.environ.get("DMLAB_MERGE_PIPE", "1") != "0"))
                    and H % 2 == 0 and W % 2 == 0
                    and os.environ.get("DMLAB_MERGE_SHORTCUT", "1") != "0"):
                dy2, wd2 = shortcut["join"]()
                if (dy2.shape[:3] == dy.shape[:3] and dy2.shape[3] % 64 == 0
                        and (cfg in _MULTI_IGEMM or dy2.shape[3] == dy.shape[3])):
                    merge_kw = dict(dy2=dy2, wd2=wd2)
                    shortcut["merged"] = True
            red_kw = (_dgrad_red(L, red_for, cfg, s, dx, complete_s2=bool(merge_kw))
                      if red_for is not None else {})
            if isinstance(dx_add, tuple):
                L.conv_dgrad(dy, wd, dx, k, k, s, p, dx_add[1], cfg, add_mask=dx_add[2], **red_kw,
                             **bwd_kw)
            else:
                L.conv_dgrad(dy, wd, dx, k, k, s, p, dx_add, cfg, **red_kw, **merge_kw, **bwd_kw)
    if ctx["has_res"]:
        return dx, (("masked", dout, ctx["mask"]) if masked_res else dres)
    return dx
