"""Per-kernel sums of rocprofv3 --pmc counter CSVs (any number of passes), averaged per dispatch,
plus derived fractions: MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs over GRBM_GUI_ACTIVE / 8
XCDs), the SQ wait buckets over SQ_WAVE_CYCLES, LDS bank-conflict cycles over LDS-array cycles.

  python tools/pmc_kernels.py <counter_collection.csv> [...]
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
            per[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add((path, r.get("Dispatch_Id") or r.get("Correlation_Id")))
    out = {}
    for name, c in per.items():
        n = max(1, len(disp[name]) // max(1, len(sys.argv) - 1))
        rec = {k: round(v / n, 1) for k, v in sorted(c.items())}
        if c.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            rec["mfma_busy_frac"] = round((c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024) / (c["GRBM_GUI_ACTIVE"] / 8), 4)
        if c.get("SQ_WAVE_CYCLES"):
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if k in c:
                    rec[k.lower() + "_frac"] = round(c[k] / c["SQ_WAVE_CYCLES"], 4)
        if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c:
            rec["lds_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
        rec["dispatches"] = n
        out[name] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
