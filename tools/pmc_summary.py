"""Per-kernel-family MFMA / LDS counter summary of a rocprofv3 ``--pmc`` CSV.

    python tools/pmc_summary.py <pmc_counter_collection.csv>

MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs): the
GRBM count is summed over the 8 XCDs, the MFMA count over every SIMD (same formula as
``profiles/pmc_halo_conv_r1s2.txt``).  Families are sorted by summed kernel time.
"""
import csv
import sys
from collections import defaultdict

from prof_summary import family

SIMDS, XCDS = 1024, 8


def main(path):
    per = defaultdict(lambda: defaultdict(float))
    seen = set()
    for r in csv.DictReader(open(path)):
        f = family(r["Kernel_Name"])
        per[f][r["Counter_Name"]] += float(r["Counter_Value"])
        if (r["Dispatch_Id"]) not in seen:
            seen.add(r["Dispatch_Id"])
            per[f]["_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per[f]["_n"] += 1
    tot = sum(d["_ns"] for d in per.values())
    print(f"{'time ms':>8} {'share':>6} {'MFMA busy':>9} {'LDS confl/cyc/CU':>16}  kernel")
    for f, d in sorted(per.items(), key=lambda kv: -kv[1]["_ns"]):
        cyc = d["GRBM_GUI_ACTIVE"] / XCDS
        mfma = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS) if cyc else 0.0
        lds = d["SQ_LDS_BANK_CONFLICT"] / (cyc * SIMDS / 4) if cyc else 0.0
        print(f"{d['_ns'] / 1e6:8.3f} {d['_ns'] / tot:6.1%} {mfma:9.1%} {lds:16.3f}  {f}")


if __name__ == "__main__":
    main(sys.argv[1])
