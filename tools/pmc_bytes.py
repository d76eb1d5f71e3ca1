"""HBM traffic per kernel family from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_bytes.py <fetch pmc_counter_collection.csv> <write pmc_counter_collection.csv>

Prints GB read/written per step (5 profiled steps: --steps 3 --warmup 2) and the achieved
TB/s of each family (profiles/pmc_resnet18_b512_hbm_bytes_r2a.txt).
"""
import csv, re, sys
from collections import defaultdict
def load(path, cname):
    d = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != cname: continue
        k = r["Dispatch_Id"]
        d[k] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), d.get(k, (0,0,0))[2] + float(r["Counter_Value"]))
    return d
f = load(sys.argv[1], "FETCH_SIZE"); w = load(sys.argv[2], "WRITE_SIZE")
def fam(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("dm::", "")
    return re.sub(r"\(.*", "", n)[:55]
agg = defaultdict(lambda: [0.0, 0.0, 0.0, 0])
for k, (n, ns, v) in f.items(): a = agg[fam(n)]; a[0] += v; a[2] += ns; a[3] += 1
for k, (n, ns, v) in w.items(): agg[fam(n)][1] += v
nsteps = 5
tot_r = sum(a[0] for a in agg.values()) / nsteps / 1e6; tot_w = sum(a[1] for a in agg.values()) / nsteps / 1e6
tot_t = sum(a[2] for a in agg.values()) / nsteps / 1e6
print(f"per step: read {tot_r:.2f} GB, write {tot_w:.2f} GB, kernel time {tot_t:.2f} ms (profiled)")
print(f"{'ms/step':>8} {'rd GB':>7} {'wr GB':>7} {'TB/s':>6}  kernel")
for n, a in sorted(agg.items(), key=lambda kv: -kv[1][2])[:28]:
    ms = a[2] / nsteps / 1e6
    print(f"{ms:8.3f} {a[0]/nsteps/1e6:7.3f} {a[1]/nsteps/1e6:7.3f} {(a[0]+a[1])/nsteps/1e6/ms if ms else 0:6.2f}  {n}")
