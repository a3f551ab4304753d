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
config = int(sys.argv[2]) if len(sys.argv) > 2 else 2
root = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.getcwd()), "gpurun_out")
NMB = 120 * 68 if config == 2 else 240 * 135
# the kernels whose bytes the bench line's roofline prices (bench.py an_name)
# (config 2: k_mb_flow, the dataflow wavefront, or with JMH_FLOW=0 the tick kernels' k_mb_analyse)
ROOFLINE = {2: ["k_mb_flow", "k_mb_analyse"], 3: ["k_mb_epzs", "k_mb_intra"], 5: ["k_rdo_inter", "k_rdo_intra", "k_rdo_final"]}[config]


def bench_line():
    """the bench JSON line of the FETCH_SIZE pass (P pictures = the pipeline fill + the timed steps)"""
    with open(os.path.join(root, f"pmc_{tag}_fetch_size.log")) as f:
        for line in f:
            if line.startswith("{"):
                return json.loads(line)
    raise SystemExit("no bench line in the FETCH_SIZE pass log")


b = bench_line()
steps = b["timed_region"]["warmup_steps_run"] + b["steps"]   # P pictures encoded in total


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


out = {"tag": tag, "config": config, "pictures": {"idr": 1, "p": steps}, "kernels": {}}
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
def base_name(k):   # "void k_mb_epzs<unsigned char, false>" -> "k_mb_epzs"
    k = k.split("(")[0].split("<")[0].strip()
    return k[5:] if k.startswith("void ") else k


roof = [k for k in out["kernels"] if base_name(k) in ROOFLINE]
if config == 2 and any(base_name(k) == "k_mb_flow" for k in roof):   # the dataflow run: its one kernel
    roof = [k for k in roof if base_name(k) == "k_mb_flow"]
if roof and all("hbm_bytes_per_mb" in out["kernels"][k] for k in roof):
    out["roofline_kernels"] = roof
    out["roofline_hbm_bytes_per_mb"] = round(sum(out["kernels"][k]["hbm_bytes_per_mb"] for k in roof), 1)
    if all("insts_per_mb" in out["kernels"][k] for k in roof):   # bench.py's issue roofline
        out["roofline_valu_insts_per_mb"] = round(sum(out["kernels"][k]["insts_per_mb"]["SQ_INSTS_VALU"] for k in roof), 1)
if hbm_total:
    out["hbm_bytes_per_mb"] = round(hbm_total / mbs, 1)
    out["note"] = ("all wavefront kernels; 2 x FETCH_SIZE + WRITE_SIZE over 1 IDR + %d P pictures, per MB; "
                   "FETCH_SIZE doubled per the gfx950 correction (an upper estimate for dword/byte loads)" % steps)
print(json.dumps(out, indent=1))
