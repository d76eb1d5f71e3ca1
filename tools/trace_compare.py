"""Compare rocprofv3 kernel traces of the same training step (e.g. plain vs forced RCCL).

    python tools/trace_compare.py <dir_or_csv> [<dir_or_csv> ...]

Per trace: the hardware queue / stream of every stream that ran kernels, the mean step time
(between consecutive optimizer dispatches), per-stream kernel-busy time, and the main
stream's forward time (dispatches before the loss kernel) -- all over the last 3 steps.
"""
import collections
import csv
import glob
import os
import sys


def load(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    return sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))


def summarise(path, nsteps=3):
    rows = load(path)
    sg = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
    per_stream = collections.Counter(r["Stream_Id"] for r in rows)
    main = None
    steps, busy, fwd = [], collections.Counter(), []
    for a, b in zip(sg[-nsteps - 1:-1], sg[-nsteps:]):
        t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
        steps.append((t1 - t0) / 1e3)
        win = rows[a + 1:b + 1]
        main = rows[b]["Stream_Id"]
        f = 0
        for r in win:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            busy[r["Stream_Id"]] += d / nsteps
            if "ce_fwd_bwd" in r["Kernel_Name"]:
                f = int(r["Start_Timestamp"]) - t0
        fwd.append(f / 1e3)
    qs = sorted({(r["Queue_Id"], r["Stream_Id"]) for r in rows}, key=lambda t: int(t[1]))
    print(f"{path}: step {sum(steps) / len(steps):.0f} us ({', '.join(f'{s:.0f}' for s in steps)}), "
          f"forward {sum(fwd) / len(fwd):.0f} us, main stream {main}")
    print("   busy/step: " + ", ".join(f"s{s} {v:.0f}" for s, v in busy.most_common()))
    print("   (queue, stream): kernels " + ", ".join(f"q{q}/s{s}: {per_stream[s]}" for q, s in qs))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        summarise(p)
