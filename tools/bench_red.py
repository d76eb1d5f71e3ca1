"""Isolated cost of the BN-backward reduction epilogue (RED) on the data-gradient tiles.

For each ResNet-18 stride-1 3x3 data gradient that carries the consumer BatchNorm's Σdz,
Σdz·x̂ in its epilogue (layer 1: res64 cfg 80; layer 2: halo cfg 42; layers 3-4: pipelined
cfg 90), times the plain launch, the RED launch with the ReLU condition (y*scale + shift > 0)
and the RED launch with the 1-bit mask, interleaved in one process.

    python tools/bench_red.py [--batch 1024] [--iters 20]
"""
import argparse
import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from dmlab.ops._native import lib  # noqa: E402

# (name, H, C, cfg)
SHAPES = [("l1_3x3", 56, 64, 80), ("l2_3x3", 28, 128, 42), ("l3_3x3", 14, 256, 90),
          ("l4_3x3", 7, 512, 90)]


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    L = lib()
    for name, H, C, cfg in SHAPES:
        N = a.batch
        g = torch.Generator(device=dev).manual_seed(1)
        w = torch.randn(C, C, 3, 3, device=dev, generator=g) / math.sqrt(C * 9)
        wf = torch.empty(C, 3, 3, C, device=dev, dtype=torch.bfloat16)
        wd = torch.empty(C, 3, 3, C, device=dev, dtype=torch.bfloat16)
        L.pack_weights(w.contiguous(), wf, wd, C)
        dy = torch.randn(N, H, H, C, device=dev, generator=g).bfloat16()
        yb = torch.randn(N, H, H, C, device=dev, generator=g).bfloat16()
        out = torch.empty_like(dy)
        sc = torch.rand(C, device=dev, generator=g) + 0.5
        sh = torch.randn(C, device=dev, generator=g) * 0.5
        mu = torch.randn(C, device=dev, generator=g) * 0.2
        inv = torch.rand(C, device=dev, generator=g) + 0.5
        mask = torch.randint(0, 256, (N * H * H * C // 8,), device=dev, dtype=torch.uint8)
        rows = L.conv_stats_rows(N * H * H, cfg, C)
        part = torch.empty(rows * 2 * C, device=dev)
        red = dict(red_y=yb, red_scale=sc, red_shift=sh, red_mean=mu, red_invstd=inv, red_part=part)
        fns = {
            "plain": lambda: L.conv_dgrad(dy, wd, out, 3, 3, 1, 1, None, cfg),
            "red_relu": lambda: L.conv_dgrad(dy, wd, out, 3, 3, 1, 1, None, cfg, **red),
            "red_mask": lambda: L.conv_dgrad(dy, wd, out, 3, 3, 1, 1, None, cfg, red_mask=mask, **red),
        }
        t = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                t[k].append(timeit(f, a.iters))
        flops = 2.0 * N * H * H * C * C * 9
        res = {k: round(min(v), 1) for k, v in t.items()}
        print(json.dumps({"shape": name, "cfg": cfg, "batch": N, "us": res,
                          "tflops_plain": round(flops / res["plain"] / 1e6, 1),
                          "red_cost_us": {k: round(res[k] - res["plain"], 1)
                                          for k in ("red_relu", "red_mask")}}), flush=True)


if __name__ == "__main__":
    main()
