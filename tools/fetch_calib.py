#!/usr/bin/env python3
"""FETCH_SIZE calibration (tools/fetch_calib.hip): per load width, FETCH_SIZE (KB) x 1024 divided
by the bytes the kernel streams (1 GiB each) -> gpurun_out/fetch_calib.json.  The factor that
turns a FETCH_SIZE reading into HBM bytes for that width is 1 / ratio.
    python3 tools/fetch_calib.py gpurun_out/fetch_calib"""
import csv
import glob
import json
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fetch_calib"
vals = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if row.get("Counter_Name") != "FETCH_SIZE":
            continue
        k = row.get("Kernel_Name", "")
        if "k_read" not in k:
            continue
        width = k.split("<")[1].split(">")[0] if "<" in k else k
        vals[width] = vals.get(width, 0.0) + float(row["Counter_Value"])
n = 1 << 30
out = {"bytes_per_kernel": n, "widths": {}}
for w, v in sorted(vals.items(), key=lambda kv: int(kv[0]) if kv[0].isdigit() else 0):
    ratio = v * 1024 / n
    out["widths"][f"{w}B_per_lane"] = {"fetch_size_kb": v, "ratio": round(ratio, 4), "factor": round(1 / ratio, 4) if ratio else None}
print(json.dumps(out, indent=1))
