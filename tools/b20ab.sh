#!/bin/bash
# the driver's config-2 invocation, env knob A/B interleaved: bash tools/b20ab.sh TAG ROUNDS VAR v1 v2 ...
TAG=$1; N=$2; VAR=$3; shift 3
for i in $(seq 1 $N); do for v in "$@"; do
  env "$VAR=$v" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_${v}_$i.json 2>/dev/null || exit 1
  python - gpurun_out/${TAG}_${v}_$i.json "$VAR=$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
print(f'{sys.argv[2]} value {d["value"]}  launches/pic {r["launches_per_picture"]}  MBs/launch {r["mbs_per_launch"]}  launch ms {r["avg_launch_ms"]}  ms/step {d["ms_per_step"]}')
PY
done; done
