#!/bin/bash
# A/B of one environment knob of the library on bench.py: bench --config C --steps 60 per value,
# twice each.   usage (GPU box): bash tools/ab_env.sh TAG CONFIG VAR value1 value2 ...
TAG=$1; CFG=$2; VAR=$3; shift 3
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --config $CFG --steps 60 --no-cpu-baseline --no-host-path \
        > gpurun_out/${TAG}_${v}_$round.json 2> gpurun_out/${TAG}_${v}_$round.err || exit $?
    echo "$VAR=$v $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_${v}_$round.json | head -1) $(grep -o '"pictures_completed": \[[0-9]*\]' gpurun_out/${TAG}_${v}_$round.json)"
  done
done
