"""HBM traffic per launch of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950). Per MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB
and reads exactly half of a wide (16 B/lane or LDS-DMA) streaming read on gfx950, so it is
doubled; WRITE_SIZE (KiB) is exact for 16 B/lane stores (ours are 8 B/lane: uncalibrated,
reported as is).

  python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
      <kernel-substring> <grid-workgroups> > profiles/roofline_traffic.json
"""
import csv
import json
import sys


def per_launch(path, counter, kname, wgs):
    vals = []
    for r in csv.DictReader(open(path)):
        if kname in r["Kernel_Name"] and r["Counter_Name"] == counter:
            grid = int(r["Grid_Size"])
            wg = int(r["Workgroup_Size"])
            if grid // wg == wgs:
                vals.append(float(r["Counter_Value"]))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    fcsv, wcsv, kname, wgs = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    fetch, nf = per_launch(fcsv, "FETCH_SIZE", kname, wgs)
    write, nw = per_launch(wcsv, "WRITE_SIZE", kname, wgs)
    out = {"kernel": kname, "grid": wgs, "fetch_kib_raw": fetch, "write_kib": write, "launches": [nf, nw]}
    if fetch is not None and write is not None:
        out["bytes_per_launch"] = int((2 * fetch + write) * 1024)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
