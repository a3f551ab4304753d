#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace (--kernel-trace, CSV), by
the (previous kernel, next kernel) pair, over the full-grid ticks only (both kernels' grids within
5 % of their largest): how much of a config-2 tick is neither k_mb_analyse nor k_mb_final.
    python tools/kernel_gaps.py TRACE.csv"""
import csv
import sys
from collections import defaultdict


def short(n):
    return n.split("(")[0].split("<")[0].replace("void ", "")


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Grid_Size_X"])))
    rows.sort()
    gmax = defaultdict(int)
    for _, _, n, g in rows:
        gmax[n] = max(gmax[n], g)
    full = [r for r in rows if r[3] >= 0.95 * gmax[r[2]]]
    gaps = defaultdict(list)
    durs = defaultdict(list)
    for a, b in zip(rows, rows[1:]):
        if a in full and b in full or (a[3] >= 0.95 * gmax[a[2]] and b[3] >= 0.95 * gmax[b[2]]):
            gaps[(a[2], b[2])].append((b[0] - a[1]) / 1e3)
    for s, e, n, g in full:
        durs[n].append((e - s) / 1e3)
    print("kernel,launches_full,avg_us")
    for n, v in durs.items():
        print(f"{n},{len(v)},{sum(v) / len(v):.2f}")
    print("prev,next,count,avg_gap_us,p50_gap_us")
    for (a, b), v in sorted(gaps.items()):
        v.sort()
        print(f"{a},{b},{len(v)},{sum(v) / len(v):.2f},{v[len(v) // 2]:.2f}")


if __name__ == "__main__":
    main()
