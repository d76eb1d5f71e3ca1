"""Brief issue-mix summary of rocprofv3 --pmc passes of one kernel run (tools/conv_one.py).

    python tools/pmc_brief.py <dir_pass1> [<dir_pass2> ...]
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 XCDs x 1024 SIMDs); the SQ_WAIT_* /
SQ_ACTIVE_* counters as fractions of SQ_WAVE_CYCLES; instruction counts per MFMA.
"""
import collections
import csv
import sys


def main(dirs):
    tot = collections.defaultdict(float)
    grbm = 0.0
    for i, d in enumerate(dirs):
        for r in csv.DictReader(open(f"{d}/pmc_counter_collection.csv")):
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                if i == 0:
                    grbm += float(r["Counter_Value"])
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    wc = tot.get("SQ_WAVE_CYCLES", 0) or 1
    mf = tot.get("SQ_INSTS_MFMA", 0) or 1
    out = {}
    if grbm:
        out["mfma_busy"] = tot.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (grbm / 8 * 1024)
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
        if k in tot:
            out[k.replace("SQ_", "").lower()] = tot[k] / wc
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
        if k in tot:
            out[k.replace("SQ_INSTS_", "").lower() + "_per_mfma"] = tot[k] / mf
    if "SQ_LDS_BANK_CONFLICT" in tot and tot.get("SQ_ACTIVE_INST_LDS"):
        out["lds_conflict_per_lds_cycle"] = tot["SQ_LDS_BANK_CONFLICT"] / tot["SQ_ACTIVE_INST_LDS"]
    print(" ".join(f"{k}={v:.3f}" for k, v in out.items()))


if __name__ == "__main__":
    main(sys.argv[1:])
