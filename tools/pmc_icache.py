#!/usr/bin/env python3
"""Per kernel, from tools/pmc_icache.sh: I-cache hit rate, misses per wave, instruction fetches
per wave and the mean fetches in flight (SQ_IFETCH_LEVEL / SQ_WAVE_CYCLES), VALU / SALU per wave."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
root = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.getcwd()), "gpurun_out")
out = {}
for cfg in ("c2", "c5"):
    sums = defaultdict(float)
    for f in glob.glob(os.path.join(root, f"pmci_{tag}_{cfg}_*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            try:
                sums[(row.get("Kernel_Name", "").split("(")[0], row["Counter_Name"])] += float(row["Counter_Value"])
            except (KeyError, ValueError):
                pass
    for k in sorted({k for k, _ in sums}):
        c = {n: v for (kk, n), v in sums.items() if kk == k}
        w = c.get("SQ_WAVES") or 0
        h, m = c.get("SQC_ICACHE_HITS", 0), c.get("SQC_ICACHE_MISSES", 0)
        if not w or not (h + m):
            continue
        out.setdefault(cfg, {})[k] = {
            "icache_hit_rate": round(h / (h + m), 4), "icache_misses": m,
            "ifetch_per_wave": round(c.get("SQ_IFETCH", 0) / w, 1),
            "ifetch_in_flight_per_wave_cycle": round(c.get("SQ_IFETCH_LEVEL", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1)), 3),
            "wait_inst_any_share": round(c.get("SQ_WAIT_INST_ANY", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1)), 3),
            "valu_per_wave": round(c.get("SQ_INSTS_VALU", 0) / w, 1), "salu_per_wave": round(c.get("SQ_INSTS_SALU", 0) / w, 1),
            "waves": w}
print(json.dumps(out, indent=1))
