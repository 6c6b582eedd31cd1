"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid): launches, average and total
duration, share of GPU time. The per-grid split is what makes the bench's roofline kernel
(one GEMM template launched at many shapes) comparable with the in-bench HIP-event average.

  python tools/prof_summary.py gpurun_out/prof/<...>_kernel_trace.csv [--top 40] > profiles/x.txt
"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict


def main(path: str, top: int = 40):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(lambda: [0, 0.0])
    total = 0.0
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3  # us
        grid = tuple(r.get(k, "") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        wg = r.get("Workgroup_Size_X", "")
        key = (name[:110], grid, wg)
        agg[key][0] += 1
        agg[key][1] += dur
        total += dur
    print(f"# {len(rows)} dispatches, {total / 1e3:.2f} ms GPU time total")
    print(f"{'share':>6} {'total_ms':>9} {'count':>6} {'avg_us':>9}  grid(x,y,z)/wg  kernel")
    for (name, grid, wg), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{100 * t / total:6.2f} {t / 1e3:9.3f} {n:6d} {t / n:9.2f}  {'x'.join(grid)}/{wg}  {name}")


if __name__ == "__main__":
    top = 40
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
    main(sys.argv[1], top)
