"""Run one conv kernel configuration repeatedly (for rocprofv3 PMC collection)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from dmlab.ops._native import lib  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "l3"
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 6
shapes = {"l1": (56, 64, 64), "l2": (28, 128, 128), "l3": (14, 256, 256), "l4": (7, 512, 512)}
H, C, Co = shapes[name]
N = 256
L = lib()
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
wf = (torch.randn(Co, 3, 3, C, device="cuda") * 0.05).bfloat16()
y = torch.empty(N, H, H, Co, device="cuda", dtype=torch.bfloat16)
T = L.conv_stats_rows(N * H * H, cfg, Co)
st = torch.empty(T * 2 * Co, device="cuda")
for _ in range(10):
    L.conv_fwd(x, wf, y, st, None, 3, 3, 1, 1, cfg)
torch.cuda.synchronize()
