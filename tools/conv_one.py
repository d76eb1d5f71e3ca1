"""Run one conv kernel configuration repeatedly (for rocprofv3 PMC collection).

    python tools/conv_one.py <l1|l2|l3|l4> <cfg> [fwd|pre|dgrad] [batch]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from dmlab.ops._native import lib  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "l3"
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 6
mode = sys.argv[3] if len(sys.argv) > 3 else "fwd"
N = int(sys.argv[4]) if len(sys.argv) > 4 else 256
shapes = {"l1": (56, 64, 64), "l2": (28, 128, 128), "l3": (14, 256, 256), "l4": (7, 512, 512)}
H, C, Co = shapes[name]
L = lib()
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
wf = (torch.randn(Co, 3, 3, C, device="cuda") * 0.05).bfloat16()
y = torch.empty(N, H, H, Co, device="cuda", dtype=torch.bfloat16)
T = L.conv_stats_rows(N * H * H, cfg, Co)
st = torch.empty(T * 2 * Co, device="cuda")
kw = {}
if mode == "pre":
    kw = dict(pre_scale=torch.rand(C, device="cuda") + 0.5, pre_shift=torch.randn(C, device="cuda") * 0.1)
for _ in range(10):
    if mode == "dgrad":
        L.conv_dgrad(y, wf, x, 3, 3, 1, 1, None, cfg)
    else:
        L.conv_fwd(x, wf, y, st, None, 3, 3, 1, 1, cfg, **kw)
torch.cuda.synchronize()
