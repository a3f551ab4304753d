#!/bin/bash
# A/B of an env knob on the driver's 20-step invocation: bash ab20.sh TAG VAR v1 v2 ... (3 rounds)
TAG=$1; VAR=$2; shift 2
for r in 1 2 3; do for v in "$@"; do
  env "$VAR=$v" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_${v}_$r.json 2>/dev/null || exit 1
  echo "$VAR=$v $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_${v}_$r.json)"
done; done
