#!/bin/bash
# the driver's config-2 invocation N times: value, flow launches per picture, MBs per launch, wavefront ms / picture
TAG=$1; N=${2:-6}
for i in $(seq 1 $N); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_$i.json 2>/dev/null || exit 1
  python - gpurun_out/${TAG}_$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
print(f'value {d["value"]}  launches/pic {r["launches_per_picture"]}  MBs/launch {r["mbs_per_launch"]}  launch ms {r["avg_launch_ms"]}  wavefront ms/pic {d["kernel_ms_per_picture"]["wavefront"]}  ms/step {d["ms_per_step"]}')
PY
done
