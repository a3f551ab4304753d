#!/usr/bin/env python3
"""Summary of tools/pmc_wait.sh per kernel: shares of SQ_WAVE_CYCLES (WAIT_ANY = parked on
s_waitcnt or a barrier, WAIT_INST_ANY = issue stalls, ACTIVE_INST_ANY), active-instruction
shares, and per memory kind the mean latency (SQ_INST_LEVEL_x / SQ_INSTS_x, quad-cycles x 4 =
cycles) and the in-flight cycles per wave-cycle (SQ_INST_LEVEL_x x 4 / SQ_WAVE_CYCLES x 4)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
root = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.getcwd()), "gpurun_out")
sums = defaultdict(float)
for p in ("a", "b"):
    for f in glob.glob(os.path.join(root, f"pmcw_{tag}_{p}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            try:
                sums[(row.get("Kernel_Name", "").split("(")[0], row["Counter_Name"])] += float(row["Counter_Value"])
            except (KeyError, ValueError):
                pass
out = {"tag": tag, "kernels": {}}
for k in sorted({k for k, _ in sums}):
    c = {n: v for (kk, n), v in sums.items() if kk == k}
    w = c.get("SQ_WAVE_CYCLES", 0)
    if not w:
        continue
    r = {"wave_cycles": w, "waves": c.get("SQ_WAVES")}
    r["split"] = {n: round(c[n] / w, 3) for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if n in c}
    r["active"] = {n: round(c[n] / w, 3) for n in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA",
                                                    "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_MISC") if n in c}
    for kind in ("VMEM", "LDS", "SMEM"):
        lv, n = c.get(f"SQ_INST_LEVEL_{kind}"), c.get(f"SQ_INSTS_{kind}")
        if lv is not None and n:
            r[kind.lower()] = {"insts": n, "mean_latency_cycles": round(4 * lv / n, 1), "in_flight_per_wave_cycle": round(lv / w, 3)}
    out["kernels"][k] = r
print(json.dumps(out, indent=1))
