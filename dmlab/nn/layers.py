"""Layers of the dmlab engine.

Every layer has a PyTorch reference forward (``torch_forward``; backward via
local autograd) and a native path in :mod:`dmlab.ops` (explicit HIP kernels).
Parameter names and shapes follow ``torch.nn`` (``Conv2d.weight`` is OIHW,
``Linear.weight`` is [out, in]) so state dicts interchange with the reference
models; the native path packs its own bf16 layouts from the fp32 master.
"""
from __future__ import annotations

import contextlib
import math

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .program import Ctx, Layer


def _kaiming_uniform_(w, fan_in):
    # torch.nn default init for Conv2d/Linear (kaiming_uniform, a=sqrt(5))
    bound = 1.0 / math.sqrt(fan_in) if fan_in > 0 else 0
    gain_bound = math.sqrt(6.0 / ((1 + 5.0) * fan_in)) if fan_in > 0 else 0
    with torch.no_grad():
        w.uniform_(-gain_bound * math.sqrt(3.0) / math.sqrt(3.0), gain_bound)
    return bound


class Conv2d(Layer):
    """Conv2d (+ optional fused ReLU and 2×2 max-pool epilogue).

    ``pool=2`` fuses ``max_pool2d(relu(conv(x)), 2)`` — the LeNet stage
    (task1/pytorch/model.py:27-28) — into one native kernel that also stores a
    2-bit argmax per pooled element for backward."""

    def __init__(self, cin, cout, k, stride=1, padding=0, bias=True, relu=False, pool=1):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.padding = cin, cout, k, stride, padding
        self.relu, self.pool = relu, pool
        self.weight = nn.Parameter(torch.empty(cout, cin, k, k))
        self.bias = nn.Parameter(torch.empty(cout)) if bias else None
        fan_in = cin * k * k
        b = _kaiming_uniform_(self.weight, fan_in)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.uniform_(-b, b)

    def torch_forward(self, x):
        y = F.conv2d(x, self.weight, self.bias, self.stride, self.padding)
        if self.relu:
            y = F.relu(y)
        if self.pool > 1:
            y = F.max_pool2d(y, self.pool)
        return y

    def native_fwd(self, x, ctx, train):
        from dmlab.ops import conv as C

        return C.conv_fwd(self, x, ctx, train)

    def native_bwd(self, dy, ctx, need_dx):
        from dmlab.ops import conv as C

        return C.conv_bwd(self, dy, ctx, need_dx)


class Linear(Layer):
    """Linear (+ optional fused ReLU) on MFMA GEMM kernels."""

    def __init__(self, fin, fout, bias=True, relu=False):
        super().__init__()
        self.fin, self.fout, self.relu = fin, fout, relu
        self.weight = nn.Parameter(torch.empty(fout, fin))
        self.bias = nn.Parameter(torch.empty(fout)) if bias else None
        b = _kaiming_uniform_(self.weight, fin)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.uniform_(-b, b)

    def torch_forward(self, x):
        y = F.linear(x.flatten(1) if x.dim() > 2 else x, self.weight, self.bias)
        return F.relu(y) if self.relu else y

    def native_fwd(self, x, ctx, train):
        from dmlab.ops import linear as L

        return L.linear_fwd(self, x, ctx, train)

    def native_bwd(self, dy, ctx, need_dx):
        from dmlab.ops import linear as L

        return L.linear_bwd(self, dy, ctx, need_dx)


class Flatten(Layer):
    def torch_forward(self, x):
        return x.flatten(1)

    def native_fwd(self, x, ctx, train):
        ctx["shape"] = x.shape
        return x.reshape(x.shape[0], -1)

    def native_bwd(self, dy, ctx, need_dx):
        return dy.reshape(ctx["shape"]) if need_dx else None


class Softmax(Layer):
    """Softmax over classes — only for the MindSpore-notebook compat mode (B10)."""

    def torch_forward(self, x):
        return F.softmax(x, dim=1)

    def native_fwd(self, x, ctx, train):
        y = torch.softmax(x.float(), dim=1)
        ctx["y"] = y
        return y

    def native_bwd(self, dy, ctx, need_dx):
        y = ctx["y"]
        return y * (dy - (dy * y).sum(1, keepdim=True))


class ConvBN(Layer):
    """conv (no bias) → BatchNorm2d (train: batch stats) → [+residual] → [ReLU].

    Native path: NHWC bf16 implicit-GEMM conv on MFMA with the BN statistics
    reduced in the conv epilogue, then one fused BN-apply/residual/ReLU pass
    (SURVEY §2.5 'Extensions required by BASELINE.json')."""

    def __init__(self, cin, cout, k, stride=1, padding=0, relu=True, eps=1e-5, momentum=0.1):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.padding = cin, cout, k, stride, padding
        self.relu = relu
        self.eps, self.momentum = eps, momentum
        self.weight = nn.Parameter(torch.empty(cout, cin, k, k))
        nn.init.kaiming_normal_(self.weight, mode="fan_out", nonlinearity="relu")
        self.bn_weight = nn.Parameter(torch.ones(cout))
        self.bn_bias = nn.Parameter(torch.zeros(cout))
        self.register_buffer("running_mean", torch.zeros(cout))
        self.register_buffer("running_var", torch.ones(cout))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def torch_forward(self, x, residual=None):
        y = F.conv2d(x, self.weight, None, self.stride, self.padding)
        if self.training:
            self.num_batches_tracked.add_(1)
        y = F.batch_norm(y, self.running_mean, self.running_var, self.bn_weight, self.bn_bias,
                         self.training, self.momentum, self.eps)
        if residual is not None:
            y = y + residual
        return F.relu(y) if self.relu else y

    def native_fwd(self, x, ctx, train, residual=None, raw=False, pre=None):
        """raw: return the conv output y un-normalised (BN scale/shift left in ctx for the
        consumer); pre=(scale, shift): x is a raw conv output to be consumed as
        relu(x*scale + shift) — the BN-apply of the previous layer fused into this conv."""
        from dmlab.ops import convbn as CB

        return CB.convbn_fwd(self, x, ctx, train, residual, raw=raw, pre=pre)

    def native_bwd(self, dy, ctx, need_dx, dx_add=None, dx_into=None, fused_skip=False,
                   red_for=None, phase=0, shortcut=None):
        from dmlab.ops import convbn as CB

        return CB.convbn_bwd(self, dy, ctx, need_dx, dx_add=dx_add, dx_into=dx_into,
                             fused_skip=fused_skip, red_for=red_for, phase=phase,
                             shortcut=shortcut)


class ConvBNPool(ConvBN):
    """ConvBN (+ReLU) followed by a max-pool: the ResNet stem.  The native path fuses
    BN-apply, ReLU and the pool into one pass that never writes the BN output, and its
    backward gathers the pooled gradient on the fly (no unpooled gradient tensor)."""

    def __init__(self, cin, cout, k, stride=1, padding=0, pool_k=3, pool_s=2, pool_p=1):
        super().__init__(cin, cout, k, stride, padding, relu=True)
        self.pool_k, self.pool_s, self.pool_p = pool_k, pool_s, pool_p

    def torch_forward(self, x, residual=None):
        from dmlab.data import normalize_input

        y = super().torch_forward(normalize_input(x, self.weight.dtype))  # u8 images: ImageNet norm
        return F.max_pool2d(y, self.pool_k, self.pool_s, self.pool_p)


class BasicBlock(Layer):
    """ResNet BasicBlock: relu(bn2(conv2(relu(bn1(conv1 x)))) + shortcut(x))."""

    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = ConvBN(cin, cout, 3, stride, 1, relu=True)
        self.c2 = ConvBN(cout, cout, 3, 1, 1, relu=True)  # relu after the residual add
        self.down = ConvBN(cin, cout, 1, stride, 0, relu=False) if (stride != 1 or cin != cout) else None

    def torch_forward(self, x):
        idt = x if self.down is None else self.down.torch_forward(x)
        y = self.c1.torch_forward(x)
        return self.c2.torch_forward(y, residual=idt)

    def native_fwd(self, x, ctx, train):
        c1, c2, cd = Ctx(), Ctx(), Ctx()
        side = self._down_stream() if self.down is not None else None
        if side is not None:
            # the projection shortcut (1x1/s2 conv + BN) and c1 both read only x: run the
            # shortcut on the side stream so its small grids fill c1's tail and vice versa
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                idt = self.down.native_fwd(x, cd, train)
        else:
            idt = x if self.down is None else self.down.native_fwd(x, cd, train)
        # c1's BN-apply + ReLU is fused into c2's operand staging: relu(bn1(y1)) is never
        # written (c2's forward and weight-gradient halo kernels normalise y1 on the fly)
        y1 = self.c1.native_fwd(x, c1, train, raw=True)
        residual = idt
        if side is not None:
            x.record_stream(side)

            def residual():
                # joined only where c2's BN-apply adds the shortcut: c2's conv (which reads
                # y1, not the shortcut) no longer waits for the side stream (a 10-50 us
                # main-stream stall per projection block)
                main.wait_stream(side)
                # tensors the side stream allocated are used (and freed) on the main stream
                for t in [idt] + [v for v in cd.values() if torch.is_tensor(v)]:
                    t.record_stream(main)
                return idt
        out = self.c2.native_fwd(y1, c2, train, residual=residual, pre=(c1["scale"], c1["shift"]))
        ctx.update(c1=c1, c2=c2, cd=cd)
        return out

    def _down_stream(self):
        prog = getattr(self, "_prog", None)
        if prog is None or os.environ.get("DMLAB_DOWN_FWD_STREAM", "1") == "0":
            return None
        return prog._side_stream() if prog._native_active else None

    def native_bwd(self, dy, ctx, need_dx):
        # c2's backward returns (d_input_of_c2, d_residual); d_residual = ReLU-masked dy stays
        # unmaterialised ("masked", dy, mask): an identity skip adds dy where the forward's
        # 1-bit mask is set in c1's dgrad epilogue, a projection shortcut's BN backward reads
        # dy with that mask (its mode 4)
        # c1's BN backward sums (Σdz, Σdz·x̂ over c2's data gradient) reduce in that dgrad's
        # epilogue where the kernel supports it (layer1: csrc/conv_res64.hip RED)
        dy1, dres = self.c2.native_bwd(dy, ctx["c2"], True, fused_skip=need_dx,
                                       red_for=(self.c1, ctx["c1"]))
        # this block's input gradient is the previous block's output gradient: its c2
        # BN-backward sums reduce in the epilogue of the dgrad that produces it (Program sets
        # _bwd_next to the preceding layer)
        nxt = getattr(self, "_bwd_next", None)
        red_for = None
        if nxt is not None and isinstance(nxt[0], BasicBlock):
            red_for = (nxt[0].c2, nxt[1]["c2"])
        elif nxt is not None and isinstance(nxt[0], ConvBN):  # the stem
            red_for = nxt
        if self.down is None:
            # identity skip: its gradient is added in c1's dgrad epilogue (no extra pass)
            return self.c1.native_bwd(dy1, ctx["c1"], need_dx, dx_add=dres if need_dx else None,
                                      red_for=red_for)
        aux = self._bn_stream() if need_dx else None
        cd = ctx["cd"]
        if need_dx:
            # the shortcut's BN backward (reduce + apply: memory-bound passes over the block's
            # output gradient) only needs dres: with an aux stream it runs on that second
            # high-priority stream next to c1's BN backward instead of after it
            main = torch.cuda.current_stream()
            if aux is not None:
                aux.wait_stream(main)
            with torch.cuda.stream(aux) if aux is not None else contextlib.nullcontext():
                self.down.native_bwd(dres, cd, need_dx, phase=1)

            def join():
                if aux is not None:
                    main.wait_stream(aux)
                dy2 = cd["_bn_out"][0]
                dy2.record_stream(main)
                from dmlab.ops.convbn import packed_weights

                return dy2, packed_weights(self.down, need_wd=True)[1]

            # c1's stride-2 data gradient takes the shortcut's 1x1/s2 data gradient as a second
            # K segment of its parity class (0,0): dx is written once, complete, and the
            # previous block's BN-backward sums reduce in the same epilogue
            sc = {"join": join, "merged": False}
            dx = self.c1.native_bwd(dy1, ctx["c1"], need_dx, shortcut=sc, red_for=red_for)
            if sc["merged"]:
                self.down.native_bwd(dres, cd, False, phase=2)  # its weight gradient only
                return dx
            if aux is not None:
                main.wait_stream(aux)
            self.down.native_bwd(dres, cd, need_dx, dx_into=dx, phase=2)
            return dx
        self.c1.native_bwd(dy1, ctx["c1"], need_dx)
        self.down.native_bwd(dres, cd, need_dx)
        return None

    def _bn_stream(self):
        prog = getattr(self, "_prog", None)
        if prog is None or not prog._native_active:
            return None
        return prog._aux_stream()


class MaxPool(Layer):
    def __init__(self, k=3, stride=2, padding=1):
        super().__init__()
        self.k, self.stride, self.padding = k, stride, padding

    def torch_forward(self, x):
        return F.max_pool2d(x, self.k, self.stride, self.padding)

    def native_fwd(self, x, ctx, train):
        from dmlab.ops import pool as P

        return P.maxpool_fwd(self, x, ctx, train)

    def native_bwd(self, dy, ctx, need_dx):
        from dmlab.ops import pool as P

        return P.maxpool_bwd(self, dy, ctx, need_dx)


class GlobalAvgPool(Layer):
    def torch_forward(self, x):
        return F.adaptive_avg_pool2d(x, 1).flatten(1)

    def native_fwd(self, x, ctx, train):
        from dmlab.ops import pool as P

        return P.avgpool_fwd(self, x, ctx, train)

    def native_bwd(self, dy, ctx, need_dx):
        from dmlab.ops import pool as P

        return P.avgpool_bwd(self, dy, ctx, need_dx)
