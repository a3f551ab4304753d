# A/B of the 16-bit EPZS window margin (EOFF_L16) for config 5: the default build and
# h264-jm-commentary_amd/csrc/ab/libjmhip_wN.so variants (built with -DEOFF_L16=N)
set -e
for w in ${WINDOWS:-default 52 44 32}; do
  if [ $w = default ]; then L=""; else L="$GRAFT_REPO_ROOT/h264-jm-commentary_amd/csrc/ab/libjmhip_w$w.so"; fi
  JMH_LIB_PATH=$L timeout -k 10 300 python bench.py --config 5 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/ab_w$w.json 2> gpurun_out/ab_w$w.err
  echo "w$w $(grep -o '"value": [0-9.]*' gpurun_out/ab_w$w.json)"
done
