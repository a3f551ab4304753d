# A/B of bench.py for one config: bench --config C --steps 60 per variant library in csrc/ab/
# (base = the in-tree build), twice each.   usage (GPU box): bash tools/ab_cfg.sh TAG CONFIG variant...
set -e
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for round in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L="$R/h264-jm-commentary_amd/csrc/ab/libjmhip_$v.so"; fi
    JMH_LIB_PATH=$L timeout -k 10 240 python bench.py --config $CFG --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err
    echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_$v.json | head -1) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/${TAG}_$v.json | head -1)"
  done
done
