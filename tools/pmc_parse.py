#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc_traffic.sh) per kernel: counter totals, per-launch
averages, and HBM bytes per macroblock of the pipelined stream (1 IDR + STEPS P pictures).

HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB units in rocprofv3): FETCH_SIZE reads half the bytes
of streaming reads on gfx950 at every load width (1, 2, 4 and 16 B per lane, tools/fetch_calib.hip,
profiles/r5n_fetch_calib.json), WRITE_SIZE the bytes written (MI355X guide).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30       # P pictures encoded in total (warmup + timed)
root = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.getcwd()), "gpurun_out")
NMB = 120 * 68


def load(kind):
    sums, ids = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(root, f"pmc_{tag}_{kind}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "").split("(")[0]
            name = row.get("Counter_Name", "")
            try:
                v = float(row.get("Counter_Value", "0"))
            except ValueError:
                continue
            sums[(k, name)] += v
            ids[(k, name)].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    return {key: (sums[key], len(ids[key])) for key in sums}


out = {"tag": tag, "pictures": {"idr": 1, "p": steps}, "kernels": {}}
for kind in ("fetch_size", "write_size", "sq_wave_cycles", "sq_insts_valu"):
    for (k, name), (s, n) in load(kind).items():
        out["kernels"].setdefault(k, {})[name] = {"total": s, "per_launch": s / max(1, n), "launches": n}
mbs = NMB * (steps + 1)
hbm_total = 0.0
for k, cs in out["kernels"].items():
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        b = 2 * cs["FETCH_SIZE"]["total"] * 1024 + cs["WRITE_SIZE"]["total"] * 1024
        cs["hbm_bytes_per_mb"] = round(b / mbs, 1)
        hbm_total += b
    if "SQ_WAVE_CYCLES" in cs:
        w = cs["SQ_WAVE_CYCLES"]["total"]
        cs["wave_cycle_split"] = {n: round(cs[n]["total"] / w, 3) for n in
                                  ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY") if n in cs}
    if "SQ_INSTS_VALU" in cs:
        cs["insts_per_mb"] = {n: round(cs[n]["total"] / mbs, 1) for n in
                              ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU") if n in cs}
if hbm_total:
    out["hbm_bytes_per_mb"] = round(hbm_total / mbs, 1)
    out["note"] = ("all wavefront kernels; 2 x FETCH_SIZE + WRITE_SIZE over 1 IDR + %d P pictures, per MB; "
                   "FETCH_SIZE doubled per the gfx950 correction (an upper estimate for dword/byte loads)" % steps)
print(json.dumps(out, indent=1))
