"""Per-kernel sums of one or more rocprofv3 --pmc passes (counter_collection.csv files),
with derived per-wave instruction counts and wait fractions.

    python tools/pmc_kernels.py <pass_dir> [<pass_dir> ...] [--match substr]
"""
import csv
import re
import sys
from collections import defaultdict


def main(argv):
    match = None
    if "--match" in argv:
        i = argv.index("--match")
        match = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    tot = defaultdict(lambda: defaultdict(float))
    waves = defaultdict(float)
    for d in argv:
        seen = set()
        for r in csv.DictReader(open(f"{d}/pmc_counter_collection.csv")):
            n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("dm::", ""))[:60]
            if match and match not in n:
                continue
            tot[n][r["Counter_Name"]] += float(r["Counter_Value"])
            key = (n, r["Dispatch_Id"])
            if key not in seen and d == argv[0]:
                seen.add(key)
                gs = int(r.get("Grid_Size", 0) or 0)
                wg = int(r.get("Workgroup_Size", 0) or 0)
                waves[n] += gs / 64 if gs else 0
    for n, c in tot.items():
        w = waves[n] or 1
        print(f"== {n}  (waves {w:.0f})")
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        for k, v in sorted(c.items()):
            extra = ""
            if k.startswith("SQ_INSTS"):
                extra = f"  per-wave {v / w:10.1f}"
            if k.startswith("SQ_WAIT") or k.startswith("SQ_ACTIVE"):
                extra = f"  frac-wave-cycles {v / wc:6.3f}"
            print(f"  {k:28s} {v:16.0f}{extra}")


if __name__ == "__main__":
    main(sys.argv[1:])
