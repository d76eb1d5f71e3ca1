"""Summarise a rocprofv3 kernel-stats CSV into per-step times (ms) per kernel family."""
import csv
import re
import sys
from collections import defaultdict

path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
fam = defaultdict(float)
tot = 0.0
for r in rows:
    n = r["Name"]
    key = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))
    key = re.sub(r"<.*>", lambda m: m.group(0)[:40], key)
    t = float(r["TotalDurationNs"]) / 1e6 / steps
    fam[key] += t
    tot += t
for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
    if v > 0.01:
        print(f"{v:8.3f} ms  {100 * v / tot:5.1f}%  {k}")
print(f"{tot:8.3f} ms  total GPU kernel time per step")
