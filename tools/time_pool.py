"""Time the fused stem BN+ReLU+max-pool kernel at the ResNet-18 batch-512 shape.

    python tools/time_pool.py
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from dmlab.ops._native import lib  # noqa: E402

N, H, C = 512, 112, 64
dev = torch.device("cuda")
y = torch.randn(N, H, H, C, device=dev).bfloat16()
sc = torch.rand(C, device=dev) + 0.5
sh = torch.randn(C, device=dev) * 0.5
OH = (H - 1) // 2 + 1
out = torch.empty(N, OH, OH, C, device=dev, dtype=torch.bfloat16)
idx = torch.empty(N, OH, OH, C, device=dev, dtype=torch.uint8)
yarg = torch.empty_like(out)
for _ in range(3):
    lib().bn_relu_maxpool(y, sc, sh, out, idx, 3, 2, 1, yarg=yarg)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
it = 20
e0.record()
for _ in range(it):
    lib().bn_relu_maxpool(y, sc, sh, out, idx, 3, 2, 1, yarg=yarg)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / it * 1e3
gb = (y.numel() * 2 + out.numel() * 2 * 2 + idx.numel()) / 1e9
print(f"bn_relu_maxpool {us:.1f} us, {gb / us * 1e6 / 1e3:.2f} TB/s (min bytes {gb:.2f} GB)")
