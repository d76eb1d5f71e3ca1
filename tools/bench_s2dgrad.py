"""Tile sweep of the merged stride-2 data gradient (3x3/s2 conv + the block's 1x1/s2
projection as a second K segment of parity class (0,0), with the previous block's BN-backward
reduction in the epilogue) at the ResNet-18 projection-block shapes, interleaved per round.

    python tools/bench_s2dgrad.py [--batch 1024] [--iters 10] [--rounds 3]
"""
import argparse
import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from dmlab.ops._native import lib  # noqa: E402
from dmlab.ops.convbn import _cpad, dgrad_cfg  # noqa: E402

# (name, input H, Cin, Cout)
SHAPES = [("l2_s2", 56, 64, 128), ("l3_s2", 28, 128, 256), ("l4_s2", 14, 256, 512)]
WIDTH = {12: 128, 15: 128, 90: 256, 91: 128, 92: 128, 93: 64}


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def pack(L, dev, w):
    cout, cin, k, _ = w.shape
    wf = torch.empty(cout, k, k, _cpad(cin), device=dev, dtype=torch.bfloat16)
    wd = torch.empty(cin, k, k, cout, device=dev, dtype=torch.bfloat16)
    L.pack_weights(w.contiguous(), wf, wd, _cpad(cin))
    return wd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--cfgs", default="11,12,13,14,15,16,17,90,91,92,93")
    ap.add_argument("--variants", action="store_true", help="default tile: plain / merged / +RED")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    L = lib()
    for name, H, Cin, Cout in SHAPES:
        N, OH = a.batch, H // 2
        g = torch.Generator(device=dev).manual_seed(3)
        wd1 = pack(L, dev, torch.randn(Cout, Cin, 3, 3, device=dev, generator=g) / math.sqrt(9 * Cin))
        wd2 = pack(L, dev, torch.randn(Cout, Cin, 1, 1, device=dev, generator=g) / math.sqrt(Cin))
        dy1 = torch.randn(N, OH, OH, Cout, device=dev, generator=g).bfloat16()
        dy2 = torch.randn(N, OH, OH, Cout, device=dev, generator=g).bfloat16()
        yb = torch.randn(N, H, H, Cin, device=dev, generator=g).bfloat16()
        dx = torch.empty(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        mask = torch.randint(0, 256, (N * H * H * Cin // 8,), device=dev, dtype=torch.uint8)
        vec = [torch.rand(Cin, device=dev, generator=g) + 0.5 for _ in range(4)]
        cfgs = [int(c) for c in a.cfgs.split(",") if Cin % WIDTH.get(int(c), 64) == 0]
        fns = {}
        if a.variants:  # the default tile alone: plain / + merged projection / + reduction
            cfg = dgrad_cfg(N * H * H, Cin, 3, 2, Cout, H, H)
            rows = L.dgrad_s2_red_rows(N, H, H, cfg)
            part = torch.empty(rows * 2 * Cin, device=dev)
            red = dict(red_y=yb, red_scale=vec[0], red_shift=vec[1], red_mean=vec[2],
                       red_invstd=vec[3], red_part=part, red_mask=mask)
            fns = {
                "plain": lambda: L.conv_dgrad(dy1, wd1, dx, 3, 3, 2, 1, None, cfg),
                "merged": lambda: L.conv_dgrad(dy1, wd1, dx, 3, 3, 2, 1, None, cfg, dy2=dy2, wd2=wd2),
                "merged_red": lambda: L.conv_dgrad(dy1, wd1, dx, 3, 3, 2, 1, None, cfg, dy2=dy2,
                                                   wd2=wd2, **red),
            }
            cfgs = []
        for cfg in cfgs:
            rows = L.dgrad_s2_red_rows(N, H, H, cfg)
            part = torch.empty(rows * 2 * Cin, device=dev)
            red = dict(red_y=yb, red_scale=vec[0], red_shift=vec[1], red_mean=vec[2],
                       red_invstd=vec[3], red_part=part, red_mask=mask)

            def f(cfg=cfg, red=red):
                L.conv_dgrad(dy1, wd1, dx, 3, 3, 2, 1, None, cfg, dy2=dy2, wd2=wd2, **red)
            try:
                f()
                torch.cuda.synchronize()
                fns[cfg] = f
            except RuntimeError as e:  # tile refuses the geometry
                print(json.dumps({"shape": name, "cfg": cfg, "refused": str(e)[:80]}), flush=True)
        t = {c: [] for c in fns}
        for _ in range(a.rounds):
            for c, f in fns.items():
                t[c].append(timeit(f, a.iters))
        flops = 2.0 * N * OH * OH * Cout * Cin * 10  # 9 taps + the 1x1
        res = {c: round(min(v), 1) for c, v in t.items()}
        if a.variants:
            print(json.dumps({"shape": name, "cfg": dgrad_cfg(N * H * H, Cin, 3, 2, Cout, H, H),
                              "us": res}), flush=True)
            continue
        print(json.dumps({"shape": name, "default_cfg": dgrad_cfg(N * H * H, Cin, 3, 2, Cout, H, H),
                          "us": res, "tflops": {c: round(flops / v / 1e6, 1) for c, v in res.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
