set -e
for v in prio noprio prio noprio; do
  if [ $v = prio ]; then L=""; else L="$GRAFT_REPO_ROOT/h264-jm-commentary_amd/csrc/ab/libjmhip_noprio.so"; fi
  JMH_LIB_PATH=$L timeout -k 10 300 python bench.py --config 5 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.json)"
done
JMH_BLOCK_PROF=1200 timeout -k 10 300 python bench.py --config 5 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/ab_prio_bp.json 2> gpurun_out/ab_prio_bp.err
grep jmh_blocks gpurun_out/ab_prio_bp.err
