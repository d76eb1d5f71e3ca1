"""Conditioning probe for the model-level fused-stem test (tests/test_stem_fused.py).

For a few (batch, image size) configs: the fused-vs-s2d stem difference of every non-stem
gradient (e) next to the s2d path's own sensitivity to a 2^-8 input perturbation (base).
Prints per config the largest e, the largest e/base and the median base, so the test's
bound can be set from measurements rather than guessed.

    python tools/stem_cond.py
"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402


def main():
    from dmlab.models import ResNet18
    from dmlab.nn import cross_entropy
    dev = torch.device("cuda:0")
    for B, S in ((8, 64), (32, 64), (64, 64), (32, 112)):
        torch.manual_seed(4)
        a = ResNet18(num_classes=10).to(dev)
        x = torch.rand(B, 3, S, S, device=dev)
        y = torch.randint(0, 10, (B,), device=dev)
        xp = x * (1 + 2 ** -8 * torch.randn_like(x))

        def run(fused, xx):
            os.environ["DMLAB_STEM_FUSED"] = fused
            a.flat.grad.zero_()
            loss = cross_entropy(a(xx), y)
            loss.backward()
            torch.cuda.synchronize()
            return loss.item(), {n: p.grad.detach().clone() for n, p in a.named_parameters()}

        (la, ga), (lb, gb), (_, gp) = run("1", x), run("0", x), run("0", xp)
        rows = []
        for n in ga:
            if n.startswith("stem."):
                continue
            d = (gb[n].norm() + 1e-12)
            rows.append((n, ((ga[n] - gb[n]).norm() / d).item(), ((gp[n] - gb[n]).norm() / d).item()))
        es = sorted(r[1] for r in rows)
        bs = sorted(r[2] for r in rows)
        worst = max(rows, key=lambda r: r[1] / (r[2] + 1e-6))
        print(json.dumps({"batch": B, "size": S, "loss": [la, lb], "max_e": es[-1], "median_e": es[len(es) // 2],
                          "max_base": bs[-1], "median_base": bs[len(bs) // 2],
                          "worst_ratio": [worst[0], worst[1], worst[2]]}), flush=True)


if __name__ == "__main__":
    main()
