"""hipBLASLt (torch.mm) throughput on the implicit-GEMM shapes of every ResNet-18 conv:
the library ceiling a plain GEMM of the same M x N x K reaches (no im2col gather)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from tools.bench_conv import EXTRA, SHAPES, timeit  # noqa: E402


def main():
    N = 256
    for name, H, C, Co, k, s, p in SHAPES + EXTRA:
        OH = (H + 2 * p - k) // s + 1
        M, K = N * OH * OH, k * k * C
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(K, Co, device="cuda").bfloat16()
        bt = torch.randn(Co, K, device="cuda").bfloat16().t()
        fl = 2.0 * M * Co * K
        t1 = timeit(lambda: torch.mm(a, b), 30)
        t2 = timeit(lambda: torch.mm(a, bt), 30)
        print(json.dumps({"shape": name, "M": M, "N": Co, "K": K,
                          "mm_TF": round(fl / t1 / 1e12, 1), "mm_bt_TF": round(fl / t2 / 1e12, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
