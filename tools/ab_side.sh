# A/B: k_rdo_intra on a side stream beside k_rdo_inter (default) vs after it (JMH_RDO_SIDE=0)
set -e
timeout -k 10 300 python -u -m pytest tests/test_rdo_gpu.py tests/test_epzs_jm10.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5s_tests.log 2>&1
tail -1 gpurun_out/r5s_tests.log
for side in 1 0 1; do
  JMH_RDO_SIDE=$side timeout -k 10 300 python bench.py --config 5 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/r5s_side$side.json 2> gpurun_out/r5s_side$side.err
  echo "side=$side $(grep -o '"value": [0-9.]*' gpurun_out/r5s_side$side.json)"
done
