"""Micro-benchmark of the implicit-GEMM conv kernels on every ResNet-18 layer shape.

Interleaves variants in one process (methodology: cdna guide §5.4 rule 24) and
prints TFLOP/s per (shape, pass, variant); checks that variants agree numerically.

    python tools/bench_conv.py [--batch 256] [--iters 20]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from dmlab.ops._native import lib  # noqa: E402

# (name, H_in, Cin, Cout, k, stride, pad)
SHAPES = [
    ("stem7x7", 224, 8, 64, 7, 2, 3),
    # the stem as run: 4x4/s1 conv over the space-to-depth input (16 ch, 112x112, output
    # 112x112: pad 2 top/left, the 113th row/column is never computed)
    ("stem_s2d", 112, 16, 64, 4, 1, 2),
    ("l1_3x3", 56, 64, 64, 3, 1, 1),
    ("l2_3x3s2", 56, 64, 128, 3, 2, 1),
    ("l2_3x3", 28, 128, 128, 3, 1, 1),
    ("l2_down", 56, 64, 128, 1, 2, 0),
    ("l3_3x3s2", 28, 128, 256, 3, 2, 1),
    ("l3_down", 28, 128, 256, 1, 2, 0),
    ("l3_3x3", 14, 256, 256, 3, 1, 1),
    ("l4_3x3s2", 14, 256, 512, 3, 2, 1),
    ("l4_down", 14, 256, 512, 1, 2, 0),
    ("l4_3x3", 7, 512, 512, 3, 1, 1),
]
# plain GEMMs through the same kernels (1x1 conv, K = C): structure ceiling without im2col
EXTRA = [
    ("gemm_k2048_n256", 14, 2048, 256, 1, 1, 0),
    ("gemm_k1024_n512", 7, 1024, 512, 1, 1, 0),
]


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cfgs", default="15,13,39,41,42,90,91")
    ap.add_argument("--wcfgs", default="v2,h9,h3")
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    ap.add_argument("--pre", action="store_true", help="also time the fused pre-BN forward")
    ap.add_argument("--shapes", default="", help="comma list of shape names (default: ResNet-18)")
    ap.add_argument("--smul", default="1", help="comma list of multipliers of the planned "
                    "wgrad m-split S (halo variants h9/h3)")
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    N = a.batch
    cfgs = [int(c) for c in a.cfgs.split(",")]
    out = []
    shapes = SHAPES + EXTRA if a.shapes else SHAPES
    if a.shapes:
        shapes = [sh for sh in shapes if sh[0] in a.shapes.split(",")]
    for name, H, C, Co, k, s, p in shapes:
        OH = H if name == "stem_s2d" else (H + 2 * p - k) // s + 1
        flops = 2.0 * N * OH * OH * Co * k * k * C
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        wf = (torch.randn(Co, k, k, C, device=dev) * 0.05).bfloat16()
        wd = (torch.randn(C, k, k, Co, device=dev) * 0.05).bfloat16()
        y = torch.empty(N, OH, OH, Co, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(N, OH, OH, Co, device=dev).bfloat16()
        dx = torch.empty(N, H, H, C, device=dev, dtype=torch.bfloat16)
        row = {"shape": name, "gflop": round(flops / 1e9, 1)}
        if "fwd" in a.passes:
            ref = None
            for cfg in cfgs:
                if cfg in (9, 12, 15, 42) and Co % 128:
                    continue
                if cfg == 60 and name != "stem_s2d":
                    continue
                if cfg == 80 and (C, Co, k, s) != (64, 64, 3, 1):
                    continue
                M = N * OH * OH
                T = L.conv_stats_rows(M, cfg, Co)
                st = torch.empty(T * 2 * Co, device=dev)
                t = timeit(lambda: L.conv_fwd(x, wf, y, st, None, k, k, s, p, cfg), a.iters)
                row[f"fwd_c{cfg}_TF"] = round(flops / t / 1e12, 1)
                if a.pre and cfg in (39, 41, 42, 80, 90, 91, 92, 93):
                    sc = torch.rand(C, device=dev) + 0.5
                    sh = torch.randn(C, device=dev) * 0.1
                    t = timeit(lambda: L.conv_fwd(x, wf, y, st, None, k, k, s, p, cfg,
                                                  pre_scale=sc, pre_shift=sh), a.iters)
                    row[f"fwdpre_c{cfg}_TF"] = round(flops / t / 1e12, 1)
                    L.conv_fwd(x, wf, y, st, None, k, k, s, p, cfg)
                if ref is None:
                    ref = y.clone()
                else:
                    row[f"fwd_c{cfg}_maxdiff"] = float((y.float() - ref.float()).abs().max())
        if "dgrad" in a.passes and not name.startswith("stem"):
            ref = None
            for cfg in cfgs:
                if cfg in (9, 12, 15, 42) and C % 128:
                    continue
                if cfg in (60, 80) and (C, Co, k, s) != (64, 64, 3, 1):
                    continue
                t = timeit(lambda: L.conv_dgrad(dy, wd, dx, k, k, s, p, None, cfg), a.iters)
                row[f"dgrad_c{cfg}_TF"] = round(flops / t / 1e12, 1)
                if ref is None:
                    ref = dx.clone()
                else:
                    row[f"dgrad_c{cfg}_maxdiff"] = float((dx.float() - ref.float()).abs().max())
        if "wgrad" in a.passes:
            from dmlab.ops.convbn import _wgrad_plan

            M = N * OH * OH
            K = k * k * C
            dw = torch.empty(Co, C, k, k, device=dev)
            ref = None
            variants = [(v, m) for v in a.wcfgs.split(",") for m in
                        ([float(x) for x in a.smul.split(",")] if v in ("h9", "h3", "w6", "g2", "g3") else [1.0])]
            for v, mul in variants:
                force = {"v2": None, "h9": 4, "h3": 5, "w6": 6, "q8": 8, "g2": 2, "g3": 3}[v]
                if force is None:
                    c, S = _wgrad_plan(M, Co, K)
                elif force == 8:
                    if (C, Co, k, s) != (64, 64, 3, 1):
                        continue
                    c, S = _wgrad_plan(M, Co, K, k, s, C, force=8, W=OH, rows=N * OH)
                else:
                    c, S = _wgrad_plan(M, Co, K, k, s, C, force=force)
                    S = max(1, int(S * mul))
                tag = v if mul == 1.0 else f"{v}x{mul:g}"
                slab = torch.empty(S * Co * K, device=dev)
                t = timeit(lambda: L.conv_wgrad(x, dy, dw, slab, C, k, k, s, p, 0.0, S, c, False), a.iters)
                row[f"wgrad_{tag}_TF"] = round(flops / t / 1e12, 1)
                row[f"wgrad_{tag}_S"] = S
                if ref is None:
                    ref = dw.clone()
                else:
                    row[f"wgrad_{tag}_reldiff"] = float((dw - ref).norm() / ref.norm())
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
