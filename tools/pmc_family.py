"""HBM traffic and MFMA utilisation of one kernel instantiation, aggregated over all of its
dispatches in the profiled step(s), from three rocprofv3 --pmc passes (one counter group each;
FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950):

  FETCH_SIZE (KiB; on gfx950 it reads half of a wide 16 B/lane or LDS-DMA streaming read, so it
  is doubled -- MI355X_MICROARCH.md §HBM), WRITE_SIZE (KiB), and
  SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE + SQ_WAVE_CYCLES + SQ_WAIT_ANY + SQ_WAIT_INST_ANY.

MFMA busy fraction = (SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs) / (GRBM_GUI_ACTIVE / 8 XCDs),
summed over the dispatches (time-weighted).

  python tools/pmc_family.py <fetch.csv> <write.csv> <sq.csv> "<kernel name>[||<kernel name>...]" <workload key> > records.json

(one record per kernel name; several names give a JSON list)

The record (keyed by workload and kernel) goes into profiles/roofline_traffic.json's "records",
which bench.py reads for the same (workload, kernel) pair only.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def name_pattern(kname):
    """kname as a regex: "<MODE>" matches every epilogue-mode instantiation of a kernel, "*" one
    integer template argument (bench.gemm_kernel_name's EPI wildcard)"""
    kname = kname.split(" M-split")[0]  # bench's family suffix: the head rows' kernel is the one profiled
    pat = re.escape(kname).replace(re.escape("<MODE>"), r"<\d+>").replace(re.escape("*"), r"\d+")
    return re.compile(pat)


def per_dispatch(path, kname):
    """counters per dispatch of the kernel whose name (template arguments as rocprofv3 prints
    them) matches kname (name_pattern)"""
    d = defaultdict(dict)
    pat = name_pattern(kname)
    for r in csv.DictReader(open(path)):
        if pat.search(r["Kernel_Name"]):
            key = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(d))
            d[key][r["Counter_Name"]] = d[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return d


def main():
    fcsv, wcsv, scsv, knames = sys.argv[1:5]
    workload = sys.argv[5] if len(sys.argv) > 5 else "config3-full"
    recs = [record(fcsv, wcsv, scsv, k, workload) for k in dict.fromkeys(knames.split("||"))]
    print(json.dumps(recs[0] if len(recs) == 1 else recs, indent=1))


def record(fcsv, wcsv, scsv, kname, workload):
    f, w, q = per_dispatch(fcsv, kname), per_dispatch(wcsv, kname), per_dispatch(scsv, kname)
    fetch = [v["FETCH_SIZE"] for v in f.values() if "FETCH_SIZE" in v]
    write = [v["WRITE_SIZE"] for v in w.values() if "WRITE_SIZE" in v]
    out = {"workload": workload, "kernel": kname, "dispatches": [len(fetch), len(write), len(q)]}
    if fetch and write:
        out["fetch_kib_per_launch_raw"] = sum(fetch) / len(fetch)
        out["write_kib_per_launch"] = sum(write) / len(write)
        out["bytes_per_launch"] = int((2 * out["fetch_kib_per_launch_raw"] + out["write_kib_per_launch"]) * 1024)
    if q:
        busy = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for v in q.values())
        gui = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in q.values())
        wave = sum(v.get("SQ_WAVE_CYCLES", 0.0) for v in q.values())
        if gui:
            out["mfma_busy_frac"] = round((busy / 1024) / (gui / 8), 4)
        if wave:
            out["sq_wait_any_frac"] = round(sum(v.get("SQ_WAIT_ANY", 0.0) for v in q.values()) / wave, 4)
            out["sq_wait_inst_any_frac"] = round(sum(v.get("SQ_WAIT_INST_ANY", 0.0) for v in q.values()) / wave, 4)
    return out


if __name__ == "__main__":
    main()
