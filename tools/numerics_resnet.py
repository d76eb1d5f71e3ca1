"""ResNet-18 training numerics at the headline shape: native bf16 kernels vs stock PyTorch.

Three copies of the same random-init ResNet-18 train on the same synthetic batches with the
same SGD-momentum optimizer (the fused flat kernel, identical for all three):

* ``native``   -- the dmlab HIP kernels (bf16 NHWC, fp32 master weights), the bench's path;
* ``autocast`` -- the same Program on the PyTorch backend under ``torch.autocast(bf16)``
                  (stock MIOpen/hipBLASLt bf16: what a stock user would run);
* ``fp32``     -- the PyTorch backend in fp32 (the numerical reference).

Per step it records the three losses; at the end the per-layer gradient norms of the last
step and the BatchNorm running statistics.  The native path is within the stock-bf16
envelope when its distance to fp32 is comparable to autocast's distance to fp32.

    python tools/numerics_resnet.py --batch 1024 --steps 100 --res 224 > profiles/x.jsonl
"""
from __future__ import annotations

import argparse
import copy
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def run(batch, steps, res, nbatches=4, lr=0.1, seed=0, classes=1000, log=print, table=None):
    from dmlab.models import ResNet18
    from dmlab.nn import cross_entropy
    from dmlab.optim import SGD

    dev = torch.device("cuda", 0)
    torch.manual_seed(seed)
    nat = ResNet18(num_classes=classes).to(dev)
    models = {"native": nat}
    for k in ("autocast", "fp32"):
        m = copy.deepcopy(nat).set_backend("torch")
        m._flatten()
        models[k] = m
    opts = {k: SGD(m.parameters(), lr=lr, momentum=0.9) for k, m in models.items()}
    g = torch.Generator(device=dev).manual_seed(seed + 1)
    data = [(torch.rand(batch, 3, res, res, device=dev, generator=g)
             .contiguous(memory_format=torch.channels_last),
             torch.randint(0, classes, (batch,), device=dev, generator=g))
            for _ in range(nbatches)]
    hist = []
    for s in range(steps):
        x, y = data[s % nbatches]
        rec = {"step": s}
        for k, m in models.items():
            if k == "native":
                loss = cross_entropy(m(x), y)
            elif k == "autocast":
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = m(x)
                loss = F.cross_entropy(out.float(), y)
            else:
                loss = F.cross_entropy(m(x), y)
            opts[k].zero_grad()
            loss.backward()
            if s in (0, steps - 1):  # gradient norms of the first / last step, before the update
                rec[k + "_gnorm"] = {n: float(p.grad.float().norm())
                                     for n, p in m.named_parameters() if p.grad is not None}
            if s == 0 and table is not None:  # full step-0 gradients for the per-layer table
                table[k] = {n: p.grad.detach().float().clone()
                            for n, p in m.named_parameters() if p.grad is not None}
            opts[k].step()
            rec[k] = float(loss.detach())
        hist.append(rec)
        log(json.dumps({kk: (round(v, 5) if isinstance(v, float) else v)
                        for kk, v in rec.items() if not kk.endswith("gnorm")}))
        sys.stdout.flush()
    return models, hist


def summarize(models, hist):
    def dist(a, b):
        return max(abs(h[a] - h[b]) for h in hist)

    def gnorm_err(rec):
        out = {}
        for n in rec["fp32_gnorm"]:
            ref = rec["fp32_gnorm"][n]
            out[n] = (abs(rec["native_gnorm"][n] - ref) / max(ref, 1e-12),
                      abs(rec["autocast_gnorm"][n] - ref) / max(ref, 1e-12))
        return out

    gn, gn0 = gnorm_err(hist[-1]), gnorm_err(hist[0])
    bn = {}
    for (n, b_nat), (_, b_ac), (_, b_32) in zip(models["native"].named_buffers(),
                                                models["autocast"].named_buffers(),
                                                models["fp32"].named_buffers()):
        if b_32.is_floating_point():
            den = float(b_32.float().norm()) + 1e-12
            bn[n] = (float((b_nat.float() - b_32.float()).norm()) / den,
                     float((b_ac.float() - b_32.float()).norm()) / den)
    return {
        "max_loss_dist_native_fp32": dist("native", "fp32"),
        "max_loss_dist_autocast_fp32": dist("autocast", "fp32"),
        "max_loss_dist_native_autocast": dist("native", "autocast"),
        "final_loss": {k: hist[-1][k] for k in ("native", "autocast", "fp32")},
        "first_loss": {k: hist[0][k] for k in ("native", "autocast", "fp32")},
        "gnorm_rel_err_max": {"native": max(v[0] for v in gn.values()),
                              "autocast": max(v[1] for v in gn.values())},
        "gnorm_rel_err_median": {
            "native": sorted(v[0] for v in gn.values())[len(gn) // 2],
            "autocast": sorted(v[1] for v in gn.values())[len(gn) // 2]},
        # step 0: same weights and batch in all three, so this isolates the kernels' numerics
        # from the divergence of the trajectories
        "step0_gnorm_rel_err_max": {"native": max(v[0] for v in gn0.values()),
                                    "autocast": max(v[1] for v in gn0.values())},
        "step0_gnorm_rel_err_median": {
            "native": sorted(v[0] for v in gn0.values())[len(gn0) // 2],
            "autocast": sorted(v[1] for v in gn0.values())[len(gn0) // 2]},
        "bn_running_rel_err_max": {"native": max(v[0] for v in bn.values()),
                                   "autocast": max(v[1] for v in bn.values())},
    }


def layer_table(table):
    """Per parameter, step 0 (same weights and batch for all three): the full-tensor relative
    error ||g - g_fp32|| / ||g_fp32|| of native and autocast, and their ratio."""
    rows = []
    for n, ref in table["fp32"].items():
        den = float(ref.norm()) + 1e-30
        en = float((table["native"][n] - ref).norm()) / den
        ea = float((table["autocast"][n] - ref).norm()) / den
        rows.append({"param": n, "native_rel": round(en, 5), "autocast_rel": round(ea, 5),
                     "ratio": round(en / max(ea, 1e-12), 3)})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--nbatches", type=int, default=4)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--table", action="store_true",
                    help="print the per-parameter step-0 gradient error table (full tensors)")
    a = ap.parse_args()
    # first steps of the PyTorch backends can sit in MIOpen's kernel search for minutes at
    # b1024: keep a heartbeat on stderr so a supervising runner does not take it as hung
    import threading
    import time

    t0 = time.time()

    def beat():
        while True:
            time.sleep(20)
            print(f"[numerics] alive {time.time() - t0:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()
    table = {} if a.table else None
    models, hist = run(a.batch, a.steps, a.res, a.nbatches, a.lr, table=table)
    if table is not None:
        rows = layer_table(table)
        del table
        for r in rows:
            print(json.dumps(r), flush=True)
        med = sorted(r["native_rel"] for r in rows)[len(rows) // 2]
        meda = sorted(r["autocast_rel"] for r in rows)[len(rows) // 2]
        worst = max(rows, key=lambda r: r["native_rel"])
        print(json.dumps({"table_summary": {"median_native_rel": med, "median_autocast_rel": meda,
                                            "median_ratio": round(med / max(meda, 1e-12), 3),
                                            "worst_native": worst}}), flush=True)
    s = summarize(models, hist)
    s.update(batch=a.batch, steps=a.steps, res=a.res, lr=a.lr, nbatches=a.nbatches)
    print(json.dumps({"summary": s}), flush=True)


if __name__ == "__main__":
    main()
