#!/bin/bash
# A/B of library builds on one bench line: bash tools/ab_libs.sh TAG "bench args" lib1 lib2 ... (2 rounds;
# "base" = the in-tree libjmhip.so)
TAG=$1; ARGS=$2; shift 2
for r in 1 2; do for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = base ]; then unset JMH_LIB_PATH; else export JMH_LIB_PATH=$L; fi
  timeout -k 10 400 python bench.py $ARGS --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_${n}_$r.json 2>/dev/null || exit 1
  echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_${n}_$r.json)"
done; done
