"""Every dispatch of one training step (queue, start offset, duration, grid) from a rocprofv3
kernel trace, plus per-queue backward sums (profiles/rocprof_resnet18_b512_step_dispatches_r2a.txt).

    python tools/step_timeline.py <kernel_trace.csv>
"""
import csv, sys, re
rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], int(r["Grid_Size_X"])//int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"])) for r in csv.DictReader(open(sys.argv[1]))), key=lambda t: t[1])
starts = [i for i, r in enumerate(rows) if "pack_input_s2d" in r[0]]
a, b = starts[-2], starts[-1]
t0 = rows[a][1]
for n, s, e, q, gx, gy, gz in rows[a:b]:
    n = re.sub(r"\(.*", "", n.replace("void ", "").replace("dm::", ""))
    print(f"q{q} {(s-t0)/1e3:8.0f} {(e-s)/1e3:7.1f}  {gx}x{gy}x{gz}  {n[:60]}")
# per-queue sums in backward
import collections
fe = next(s for n, s, e, q, *_ in rows[a:b] if "ce_fwd_bwd" in n)
sums = collections.defaultdict(float); cat = collections.defaultdict(float)
for n, s, e, q, *_ in rows[a:b]:
    if s < fe: continue
    sums[q] += (e - s) / 1e3
    k = "conv" if ("conv" in n or "igemm" in n or "wgrad" in n) else ("bn" if "bn_" in n or "slab" in n else "other")
    cat[(q, k)] += (e - s) / 1e3
print(dict(sums)); print({k: round(v) for k, v in cat.items()})
