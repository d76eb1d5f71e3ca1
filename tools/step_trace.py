"""Per-kernel timeline of the last full training step in a rocprofv3 --kernel-trace CSV.

    python tools/step_trace.py <kernel_trace.csv> [--summary]
A step is delimited by consecutive optimizer (sgd) dispatches.  --summary prints per-stream
busy time and the main-stream gaps instead of the timeline.
"""
import csv
import sys


def main(path, summary):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    sg = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
    s0, s1 = sg[-2], sg[-1]
    t0 = int(rows[s0]["End_Timestamp"])
    step = rows[s0 + 1:s1 + 1]
    busy = {}
    for r in step:
        q = r.get("Stream_Id", r.get("Queue_Id", ""))
        st, en = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        busy[q] = busy.get(q, 0) + en - st
        if not summary:
            n = r["Kernel_Name"].replace("void dm::", "").replace("dm::", "").replace("(anonymous namespace)::", "")
            print(f"{st / 1e3:9.1f} {(en - st) / 1e3:7.1f} q{q} {n[:70]}")
    tot = (int(step[-1]["End_Timestamp"]) - t0) / 1e3
    print(f"step {tot:.1f} us; busy per stream (us): " + ", ".join(f"q{q} {b / 1e3:.1f}" for q, b in busy.items()))


if __name__ == "__main__":
    main(sys.argv[1], "--summary" in sys.argv)
