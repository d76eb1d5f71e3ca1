"""Run one weight-gradient configuration repeatedly (for rocprofv3 PMC collection).

    python tools/wgrad_one.py <cfg> [batch] [pre]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from dmlab.ops._native import lib  # noqa: E402
from dmlab.ops.convbn import _wgrad_plan  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
pre = len(sys.argv) > 3 and sys.argv[3] == "pre"
H, C = 56, 64
L = lib()
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
dy = torch.randn(N, H, H, C, device="cuda").bfloat16()
c, S = _wgrad_plan(N * H * H, C, 9 * C, 3, 1, C, force=cfg, W=H, rows=N * H)
slab = torch.empty(S * C * 9 * C, device="cuda")
dw = torch.empty(C, C, 3, 3, device="cuda")
kw = dict(pre_scale=torch.rand(C, device="cuda") + 0.5, pre_shift=torch.randn(C, device="cuda")) if pre else {}
for _ in range(10):
    L.conv_wgrad(x, dy, dw, slab, C, 3, 3, 1, 1, 0.0, S, c, False, **kw)
torch.cuda.synchronize()
