"""Per-dispatch view of rocprofv3 --pmc passes over one repeated workload (e.g. tools/gemm_vs_lib.py):
dispatches matched across passes by their order among the kernels that pass the name filter;
prints per (kernel, grid) group the mean counters and derived figures, with the kernel duration
and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) from the pass's own timestamps.

  python tools/pmc_dispatch.py <counter_collection.csv> [...]
"""
import csv
import json
import sys
from collections import defaultdict, OrderedDict


def load(path):
    disp = OrderedDict()
    for r in csv.DictReader(open(path)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                                    "vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]),
                                                    "lds": int(r["LDS_Block_Size"]),
                                                    "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                    "c": {}})
        d["c"][r["Counter_Name"]] = d["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(disp.values())


def short(n):
    n = n.replace("void (anonymous namespace)::", "").split("(")[0]
    return n[:70]


def main():
    passes = [load(p) for p in sys.argv[1:]]
    n = min(len(p) for p in passes)
    groups = defaultdict(lambda: defaultdict(list))
    order = []
    for i in range(n):
        key = (short(passes[0][i]["name"]), passes[0][i]["grid"])
        if key not in order:
            order.append(key)
        g = groups[key]
        for p in passes:
            d = p[i]
            for k, v in d["c"].items():
                g[k].append(v)
            g["_ns"].append(d["ns"])
            g["_vgpr"] = [d["vgpr"]]
            g["_agpr"] = [d["agpr"]]
            g["_lds"] = [d["lds"]]
            if "GRBM_GUI_ACTIVE" in d["c"]:
                g["_clk"].append(d["c"]["GRBM_GUI_ACTIVE"] / 8 / d["ns"])
    out = OrderedDict()
    for key in order:
        g = groups[key]
        m = {k: sum(v) / len(v) for k, v in g.items() if v}
        rec = {"grid": key[1], "us": round(m["_ns"] / 1e3, 1), "vgpr": m["_vgpr"], "agpr": m["_agpr"], "lds": m["_lds"]}
        if "_clk" in m:
            rec["eff_clock_ghz"] = round(m["_clk"], 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            rec["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (m["GRBM_GUI_ACTIVE"] / 8), 4)
        if "SQ_WAVE_CYCLES" in m:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if k in m:
                    rec[k.lower()[3:] + "_frac"] = round(m[k] / m["SQ_WAVE_CYCLES"], 4)
        if m.get("SQ_INSTS_MFMA", 0) > 0:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
                if k in m:
                    rec[k.lower()[9:] + "_per_mfma"] = round(m[k] / m["SQ_INSTS_MFMA"], 3)
        if "FETCH_SIZE" in m:
            rec["fetch_gb_x2"] = round(2 * m["FETCH_SIZE"] * 1024 / 1e9, 3)  # FETCH_SIZE is KiB; gfx950 x2
        if "WRITE_SIZE" in m:
            rec["write_gb"] = round(m["WRITE_SIZE"] * 1024 / 1e9, 3)
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            rec["l2_hit"] = round(m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
        if "SQ_LDS_IDX_ACTIVE" in m:
            rec["lds_active_per_mfma"] = round(m["SQ_LDS_IDX_ACTIVE"] / max(1.0, m.get("SQ_INSTS_MFMA", 1)), 3)
        out[f"{key[0]} grid {key[1]}"] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
