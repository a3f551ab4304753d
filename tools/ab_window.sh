set -e
for w in 52 40 32 24; do
  if [ $w = 52 ]; then L=""; else L="$GRAFT_REPO_ROOT/h264-jm-commentary_amd/csrc/ab/libjmhip_w$w.so"; fi
  JMH_LIB_PATH=$L timeout -k 10 300 python bench.py --config 5 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/r5r_w$w.json 2> gpurun_out/r5r_w$w.err
  echo "w$w $(grep -o '"value": [0-9.]*' gpurun_out/r5r_w$w.json)"
done
JMH_LIB_PATH=$GRAFT_REPO_ROOT/h264-jm-commentary_amd/csrc/ab/libjmhip_w24.so timeout -k 10 300 python -u -m pytest tests/test_rdo_gpu.py tests/test_epzs_jm10.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5r_w24_tests.log 2>&1
tail -1 gpurun_out/r5r_w24_tests.log
