"""Per-kernel-family clock, MFMA busy and wave-state split from one rocprofv3 PMC pass
(GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES, SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
SQ_ACTIVE_INST_ANY): profiles/pmc_resnet18_b512_waits_r2a.txt.

    python tools/pmc_waits.py <pmc_counter_collection.csv>
"""
import csv, sys, re
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
per = defaultdict(dict)
meta = {}
for r in rows:
    d = r["Dispatch_Id"]
    per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    meta[d] = (r["Kernel_Name"], int(r["Start_Timestamp"]) if "Start_Timestamp" in r else 0, int(r["End_Timestamp"]) if "End_Timestamp" in r else 0)
fam = defaultdict(lambda: defaultdict(float))
for d, c in per.items():
    n, s, e = meta[d]
    n = re.sub(r"\(.*", "", n.replace("void ", "").replace("dm::", ""))[:50]
    f = fam[n]
    f["ns"] += e - s; f["n"] += 1
    for k, v in c.items(): f[k] += v
tot = sum(f["ns"] for f in fam.values())
print(f"{'ms':>7} {'share':>6} {'GHz':>5} {'MFMA%':>6} {'wait%':>6} {'stall%':>6} {'act%':>5}  kernel")
for n, f in sorted(fam.items(), key=lambda kv: -kv[1]["ns"])[:30]:
    cyc = f["GRBM_GUI_ACTIVE"] / 8
    ghz = cyc / f["ns"] if f["ns"] else 0
    mf = f["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024) if cyc else 0
    wc = f["SQ_WAVE_CYCLES"] or 1
    print(f"{f['ns']/1e6:7.3f} {f['ns']/tot:6.1%} {ghz:5.2f} {mf:6.1%} {f['SQ_WAIT_ANY']/wc:6.1%} {f['SQ_WAIT_INST_ANY']/wc:6.1%} {f['SQ_ACTIVE_INST_ANY']/wc:5.1%}  {n}")
