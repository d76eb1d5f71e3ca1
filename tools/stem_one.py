"""Isolated fused-stem timing (forward, pool-apply, backward, weight reduce) at batch B,
224^2, for rocprofv3 kernel traces / PMC passes of the stem kernels alone.

    python tools/stem_one.py [--batch 1024] [--dtype u8|f32|bf16] [--iters 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dmlab.data import input_affine  # noqa: E402
from dmlab.ops._native import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--nimg", type=int, default=2048)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda")
    dt = {"u8": torch.uint8, "f32": torch.float32, "bf16": torch.bfloat16}[a.dtype]
    H = a.res
    g = torch.Generator(device=dev).manual_seed(0)
    raw = torch.randint(0, 256, (a.nimg, 3, H, H), device=dev, generator=g, dtype=torch.uint8)
    img = (raw if dt == torch.uint8 else (raw.float() / 255).to(dt)).contiguous(
        memory_format=torch.channels_last)
    B = a.batch
    idx = torch.randperm(a.nimg, device=dev)[:B]
    w = torch.randn(64, 3, 7, 7, device=dev) * 0.08
    gamma = torch.randn(64, device=dev)
    beta = torch.randn(64, device=dev) * 0.2
    wk = torch.empty(64, 176, device=dev, dtype=torch.bfloat16)
    L.stem_pack_weights(w, wk)
    PH = H // 4
    pext = torch.empty(B, PH, PH, 64, device=dev, dtype=torch.bfloat16)
    code = torch.empty(B, PH, PH, 32, device=dev, dtype=torch.uint8)
    code4 = torch.empty(B, PH, PH, 32, device=dev, dtype=torch.uint8)
    grid = L.stem_fused_grid(B)
    f = dict(device=dev, dtype=torch.float32)
    stats = torch.empty(grid * 128, **f)
    sc, bi = input_affine(dt)
    M = B * (H // 2) ** 2
    scale, shift, mean, invstd = (torch.empty(64, **f) for _ in range(4))
    rm, rv = torch.zeros(64, **f), torch.ones(64, **f)
    out = torch.empty_like(pext)
    gout = torch.randn(out.shape, device=dev).to(torch.bfloat16)
    part = torch.empty(L.bn_bwd_rows(pext.numel() // 64, 64) * 128, **f)
    dgamma, dbeta = torch.zeros(64, **f), torch.zeros(64, **f)
    dw = torch.zeros(64, 3, 7, 7, **f)
    work = torch.empty(L.bn_bwd_work(M, 64), **f)
    dslab = torch.empty(L.stem_bwd_slab_len(grid), **f)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    tt = [0.0] * 4
    for it in range(a.iters + 2):
        ev[0].record()
        L.stem_fwd_fused(img, idx, sc, bi, wk, gamma, pext, code, stats, grid)
        ev[1].record()
        L.bn_stats_finalize(stats, grid, float(M), gamma, beta, rm, rv, 0.1, 1e-5, scale, shift,
                            mean, invstd, torch.empty(256 * 128, **f))
        L.stem_pool_apply(pext, code, scale, shift, out, code4)
        ev[2].record()
        rows = L.bn_bwd_reduce_masked(gout, pext, mean, invstd, scale, shift, part)
        ev[3].record()
        L.stem_bwd_fused2(img, idx, sc, bi, wk, gout, code4, mean, invstd, gamma, dgamma, dbeta,
                          0.0, part, rows, dw, 0.0, work, dslab, grid)
        ev[4].record()
        torch.cuda.synchronize()
        if it >= 2:
            for k in range(4):
                tt[k] += ev[k].elapsed_time(ev[k + 1]) / a.iters
    print(f"stem B={B} {a.dtype}: fwd {tt[0]:.3f} ms  stats+apply {tt[1]:.3f} ms  "
          f"bwd-reduce {tt[2]:.3f} ms  bwd {tt[3]:.3f} ms  total {sum(tt):.3f} ms")


if __name__ == "__main__":
    main()
