#!/usr/bin/env python3
"""Average duration of a kernel over its steady-state launches, from a rocprofv3 kernel trace
(--kernel-trace, CSV): the launches whose grid is within 5 % of the largest grid of that kernel
(full ticks; the pipeline's fill / drain ticks and the bench's one-picture checks have smaller
grids).  This is the figure bench.py's live HIP-event average samples (every 8th tick of the timed
region, all of them full), so the two can be compared.
    python tools/steady_kernel_stats.py TRACE.csv [KERNEL_SUBSTRING ...]"""
import csv
import sys
from collections import defaultdict


def main():
    path, names = sys.argv[1], sys.argv[2:] or ["k_mb_analyse", "k_mb_final"]
    rows = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            for k in names:
                if k in n:
                    rows[n].append((int(r["Grid_Size_X"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    print("kernel,launches_all,avg_us_all,grid_full,launches_full,avg_us_full")
    for n, v in rows.items():
        g = max(x for x, _ in v)
        full = [d for x, d in v if x >= 0.95 * g]
        print(f'"{n}",{len(v)},{sum(d for _, d in v) / len(v) / 1e3:.2f},{g},{len(full)},{sum(full) / len(full) / 1e3:.2f}')


if __name__ == "__main__":
    main()
