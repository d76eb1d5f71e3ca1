"""Summarise rocprofv3 kernel times into per-step times (ms) per kernel family.

    python tools/prof_summary.py <kernel_stats.csv | results.db> [steps] [--last K]

Accepts the ``--stats`` CSV (``*_kernel_stats.csv``) or the SQLite database that
rocprofv3 writes by default (``*_results.db``).  With a database, ``--last K`` keeps
only the last K dispatches of the most frequent kernel family boundary, i.e. drops
warmup: the timed window is the final ``steps`` fraction of the trace.
"""
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def family(n):
    key = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))
    return re.sub(r"<.*>", lambda m: m.group(0)[:40], key)


def rows_csv(path):
    for r in csv.DictReader(open(path)):
        yield r["Name"], float(r["TotalDurationNs"]), int(r.get("Calls") or 1)


def rows_trace(path, keep_frac=None):
    rs = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                 for r in csv.DictReader(open(path))), key=lambda t: t[1])
    if keep_frac:
        rs = rs[int(len(rs) * (1 - keep_frac)):]
    for n, s, e in rs:
        yield n, float(e - s), 1


def step_rows(path):
    """(name, start, end, grid, wg) of the last complete step (between the last two
    optimizer launches) of a kernel-trace CSV."""
    rs = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                  r["Grid_Size_X"], r["Workgroup_Size_X"]) for r in csv.DictReader(open(path))),
                key=lambda t: t[1])
    idx = [i for i, r in enumerate(rs) if "sgd_kernel" in r[0]]
    return rs[idx[-2] + 1: idx[-1] + 1]


def rows_db(path, keep_frac=None):
    c = sqlite3.connect(path)
    rs = list(c.execute("select name, start, end from kernels order by start"))
    if keep_frac:
        rs = rs[int(len(rs) * (1 - keep_frac)):]
    for n, s, e in rs:
        yield n, float(e - s), 1


def main():
    args = [a for a in sys.argv[1:]]
    frac = None
    if "--frac" in args:
        i = args.index("--frac")
        frac = float(args[i + 1])
        del args[i:i + 2]
    step_mode = "--step" in args
    args = [x for x in args if x != "--step"]
    path = args[0]
    steps = float(args[1]) if len(args) > 1 else 1.0
    if step_mode:
        rs = step_rows(path)
        for n, s0, e, gx, wg in rs:
            print(f"{(e - s0) / 1e3:8.1f} us  grid {int(gx) // int(wg):6d}  {family(n)[:70]}")
        # busy time vs the step's wall span: the difference is launch gaps / idle GPU
        busy = sum(e - s0 for _, s0, e, _, _ in rs)
        span = rs[-1][2] - rs[0][1]
        print(f"{len(rs)} kernels, busy {busy / 1e6:.3f} ms, span {span / 1e6:.3f} ms, "
              f"gaps {(span - busy) / 1e6:.3f} ms")
        return
    if path.endswith(".db"):
        rows = rows_db(path, frac)
    elif "kernel_trace" in path:
        rows = rows_trace(path, frac)
    else:
        rows = rows_csv(path)
    fam = defaultdict(float)
    cnt = defaultdict(int)
    tot = 0.0
    for n, ns, calls in rows:
        t = ns / 1e6 / steps
        k = family(n)
        fam[k] += t
        cnt[k] += calls
        tot += t
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        if v > 0.01:
            print(f"{v:8.3f} ms  {100 * v / tot:5.1f}%  {cnt[k] / steps:5.1f}/step  {k}")
    print(f"{tot:8.3f} ms  total GPU kernel time per step")


if __name__ == "__main__":
    main()
