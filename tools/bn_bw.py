"""Achieved HBM bandwidth of the BatchNorm passes vs plain torch streams of the same bytes.

    python tools/bn_bw.py [--shape 256,56,56,64] [--reps 20]

Prints one JSON line per op: µs per call and TB/s of the bytes it must move.  Used to
decide whether the BN kernels (csrc/bn_pool.hip) are at the HBM roofline (~6.3 TB/s
measured float4 copy on MI355X) or latency/issue bound.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="256,56,56,64")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from dmlab.ops._native import lib

    L = lib()
    N, H, W, C = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda", 0)
    bf = dict(device=dev, dtype=torch.bfloat16)
    f32 = dict(device=dev, dtype=torch.float32)
    y = torch.randn(N, H, W, C, **bf)
    dz = torch.randn(N, H, W, C, **bf)
    out = torch.relu(torch.randn(N, H, W, C, **bf))
    o1 = torch.empty(N, H, W, C, **bf)
    o2 = torch.empty(N, H, W, C, **bf)
    nb = y.numel() * 2
    scale = torch.rand(C, **f32) + 0.5
    shift = torch.randn(C, **f32) * 0.1
    mean = torch.zeros(C, **f32)
    invstd = torch.ones(C, **f32)
    gamma = torch.ones(C, **f32)
    dg = torch.zeros(C, **f32)
    db = torch.zeros(C, **f32)
    M = N * H * W
    work = torch.empty(L.bn_bwd_work(M, C), **f32)

    def rep(name, us, tensors):
        print(json.dumps({"op": name, "shape": [N, H, W, C], "us": round(us, 2),
                          "MB": round(tensors * nb / 1e6, 1),
                          "TB/s": round(tensors * nb / us / 1e6, 2)}), flush=True)

    rep("torch sum (1R)", timeit(lambda: y.sum(), a.reps), 1)
    rep("torch copy (1R1W)", timeit(lambda: o1.copy_(y), a.reps), 2)
    rep("torch add (2R1W)", timeit(lambda: torch.add(y, dz, out=o1), a.reps), 3)
    rep("bn_apply relu (1R1W)", timeit(lambda: L.bn_apply(y, None, scale, shift, o1, True), a.reps), 2)
    rep("bn_apply res+relu (2R1W)",
        timeit(lambda: L.bn_apply(y, dz, scale, shift, o1, True), a.reps), 3)

    def bwd(mode, dres):
        return lambda: L.bn_backward(dz, out if mode == 1 else None, y, mean, invstd, gamma, dg, db,
                                     0.0, mode, scale, shift, None, None, 3, 2, 1, o1,
                                     o2 if dres else None, work)

    # reduce pass reads (dz, y[, out]); apply pass reads them again and writes dy[, dres]
    rep("bn_backward mode2 (reduce 2R + apply 2R1W)", timeit(bwd(2, False), a.reps), 5)
    rep("bn_backward mode1+dres (reduce 3R + apply 3R2W)", timeit(bwd(1, True), a.reps), 8)
    rep("bn_backward mode0 (reduce 2R + apply 2R1W)", timeit(bwd(0, False), a.reps), 5)


if __name__ == "__main__":
    main()
