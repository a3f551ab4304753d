#!/bin/bash
# A/B of libjmhip.so builds on one box: bash tools/ab_lib.sh TAG CONFIG "variant ..." [ROUNDS]
# variant "default" = the in-tree libjmhip.so, else h264-jm-commentary_amd/csrc/ab/libjmhip_<variant>.so
# (tools/fastbuild.sh with DEFS=... OUT=ab/libjmhip_<variant>.so); each run is
# bench.py --config CONFIG --steps 60 under its own time limit, variants interleaved per round.
set -e
TAG=$1; CONFIG=$2; VARS=$3; ROUNDS=${4:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    if [ $v = default ]; then L=""; else L="$R/h264-jm-commentary_amd/csrc/ab/libjmhip_$v.so"; fi
    o=gpurun_out/${TAG}_c${CONFIG}_${v}_$r
    JMH_LIB_PATH=$L timeout -k 10 300 python bench.py --config $CONFIG --steps 60 --no-cpu-baseline --no-host-path ${BENCH_EXTRA:-} > $o.json 2> $o.err
    echo "c$CONFIG $v round $r: $(grep -o '"value": [0-9.]*' $o.json)"
  done
done
