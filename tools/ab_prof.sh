#!/bin/bash
# Per-variant debug timings on the GPU box: the phase stamps of one 1080p P macroblock
# (JMH_PHASE_PROF, tools/phase_prof.py) and the block durations of one steady-state config-2 tick
# (JMH_BLOCK_PROF, bench.py).  usage: bash tools/ab_prof.sh TAG "variant ..." [MB] [TICK]
# (variant "default" = the in-tree libjmhip.so, else csrc/ab/libjmhip_<variant>.so; CFG=3/5: that
# bench config, block durations only)
set -e
TAG=$1; VARS=$2; MB=${3:-4100}; TICK=${4:-400}; CFG=${CFG:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for v in $VARS; do
  if [ $v = default ]; then L=""; else L="$R/h264-jm-commentary_amd/csrc/ab/libjmhip_$v.so"; fi
  [ $CFG = 2 ] && JMH_LIB_PATH=$L JMH_PHASE_PROF=$MB timeout -k 10 120 python tools/phase_prof.py 2> gpurun_out/${TAG}_${v}_phase.txt
  JMH_LIB_PATH=$L JMH_BLOCK_PROF=$TICK timeout -k 10 240 python bench.py --config $CFG --steps 60 --no-cpu-baseline --no-host-path \
      > gpurun_out/${TAG}_${v}_bprof.json 2> gpurun_out/${TAG}_${v}_bprof.txt
  echo "== $v"; [ $CFG = 2 ] && grep jmh_phase gpurun_out/${TAG}_${v}_phase.txt | tail -1; grep "jmh_blocks tick" gpurun_out/${TAG}_${v}_bprof.txt | head -2
done
