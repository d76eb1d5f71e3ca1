"""Drive the ASan/UBSan build of the C++ bucket reducer (csrc/reducer.cpp) through a 2-rank
gloo DDP run (tests/test_host_sanitizers.py).  argv[1]: directory holding reducer_asan*.so."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def _ddp_run(rank, ws, moddir):
    import importlib

    import torch
    import torch.nn.functional as F

    sys.path.insert(0, moddir)
    mod = importlib.import_module("reducer_asan")
    sys.modules["dmlab._C"] = mod  # DDP._build_native imports the Reducer from here
    from dmlab.models import Net
    from dmlab.optim import SGD
    from dmlab.parallel import DDP

    for comm_dtype in (None, torch.bfloat16):
        torch.manual_seed(0)
        model = Net()
        ddp = DDP(model, bucket_cap_mb=0.05, first_bucket_mb=0.01, comm_dtype=comm_dtype,
                  native=True)
        assert type(ddp._native).__module__ == "reducer_asan", type(ddp._native)
        opt = ddp.fold_average_into(SGD(model.parameters(), lr=0.1, momentum=0.9))
        g = torch.Generator().manual_seed(rank)
        for step in range(3):
            x, y = torch.rand(4, 1, 28, 28, generator=g), torch.randint(0, 10, (4,), generator=g)
            if step == 1:
                with ddp.no_sync():
                    F.cross_entropy(ddp(x), y).backward()
            opt.zero_grad()
            F.cross_entropy(ddp(x), y).backward()
            opt.step()
        assert ddp.buckets_launched == 2 * len(ddp.buckets) + len(ddp.buckets)  # 3 synced steps
        # bad arguments are rejected by the C++ checks, not by memory errors
        for bad in (lambda: ddp._native.mark_ready(10**6), lambda: ddp._native.mark_layer(-1)):
            try:
                bad()
            except RuntimeError:
                pass
            else:
                raise AssertionError("bad id accepted")
    print(f"rank {rank} ok", flush=True)


if __name__ == "__main__":
    from dist_helpers import run_dist

    run_dist(_ddp_run, 2, sys.argv[1])
    print("ok")
