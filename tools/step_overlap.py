"""Wall time vs busy time of one training step from a rocprofv3 kernel trace: step length,
union of busy intervals, summed kernel time (two-stream overlap), forward and backward spans.

    python tools/step_overlap.py <kernel_trace.csv>
"""
import csv, sys
rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"])
               for r in csv.DictReader(open(sys.argv[1]))), key=lambda t: t[1])
# step boundaries: pack_input_s2d kernel starts
starts = [i for i, r in enumerate(rows) if "pack_input_s2d" in r[0]]
for a, b in zip(starts[-4:-1], starts[-3:]):
    step = rows[a:b]
    t0, t1 = step[0][1], rows[b][1]
    # union of busy
    iv = sorted((s, e) for _, s, e, _ in step)
    busy = 0; cs, ce = iv[0]
    for s, e in iv[1:]:
        if s > ce: busy += ce - cs; cs, ce = s, e
        else: ce = max(ce, e)
    busy += ce - cs
    # forward end: first bn_bwd or ce_fwd_bwd kernel
    fe = next(r[1] for r in step if "ce_fwd_bwd" in r[0])
    tot = sum(e - s for _, s, e, _ in step)
    sgd = next(r for r in step if "sgd_kernel" in r[0])
    print(f"step {(t1-t0)/1e3:.0f} us  busy-union {busy/1e3:.0f} us  kernel-sum {tot/1e3:.0f} us  fwd {(fe-t0)/1e3:.0f} us  bwd->sgd-end {(sgd[2]-fe)/1e3:.0f} us  after-sgd {(t1-sgd[2])/1e3:.0f}  queues {sorted(set(r[3] for r in step))}")
