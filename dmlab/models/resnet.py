"""ResNet-18-shaped CNN — the BASELINE.json headline DDP benchmark model.

Not in the reference (SURVEY §2.5 "Extensions required by BASELINE.json"):
7×7/2 conv 3→64 + BN + ReLU, 3×3/2 max-pool, four stages of two BasicBlocks
(64/128/256/512 channels; stride 2 at the first block of stages 2-4 with a 1×1
conv+BN shortcut), global average pool, fc 512→num_classes (11.69 M params at
1000 classes).

Native execution is NHWC bf16 end to end: the input is accepted as a
``channels_last`` tensor (or converted once), every conv is an implicit-GEMM MFMA
kernel with the BatchNorm statistics reduced in its epilogue, and BN-apply,
residual add and ReLU are one fused pass.
"""
from __future__ import annotations

import torch

from dmlab.nn.layers import BasicBlock, ConvBNPool, GlobalAvgPool, Linear
from dmlab.nn.program import Program


class ResNet18(Program):
    # the s2d stem packing gathers a loader batch by index itself (no batch copy)
    accepts_gathered = True

    def __init__(self, num_classes: int = 1000, in_channels: int = 3,
                 widths=(64, 128, 256, 512)):
        super().__init__()
        # stem = conv7x7/s2 + BN + ReLU + maxpool3x3/s2 (one fused layer)
        self.stem = ConvBNPool(in_channels, widths[0], 7, 2, 3, pool_k=3, pool_s=2, pool_p=1)
        layers = [self.stem]
        cin = widths[0]
        for i, w in enumerate(widths):
            b1 = BasicBlock(cin, w, 1 if i == 0 else 2)
            b2 = BasicBlock(w, w, 1)
            setattr(self, f"layer{i + 1}_0", b1)
            setattr(self, f"layer{i + 1}_1", b2)
            layers += [b1, b2]
            cin = w
        self.avgpool = GlobalAvgPool()
        self.fc = Linear(widths[-1], num_classes)
        layers += [self.avgpool, self.fc]
        self.set_dtype(torch.bfloat16)
        self.build(layers)
        # conv weight gradients run on a second stream, overlapping the dgrad/BN chain
        self._uses_side_stream = True

    def prepare_native(self, x):
        if self.compute_dtype != torch.bfloat16:
            raise ValueError("the native ResNet path computes in bf16")
        # all conv weights re-packed to bf16 in one launch per weight version
        if getattr(self, "_packed_ver", None) != self._wver:
            from dmlab.nn.layers import ConvBN
            from dmlab.ops.convbn import pack_all

            pack_all(self, [m for m in self.modules() if type(m) is ConvBN])
            self._packed_ver = self._wver
