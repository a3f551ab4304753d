set -e
timeout -k 10 300 python -u -m pytest tests/test_rdo_gpu.py tests/test_epzs_jm10.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5v_tests.log 2>&1
tail -1 gpurun_out/r5v_tests.log
JMH_BLOCK_PROF=1200 JMH_PHASE_PROF=14500 timeout -k 10 300 python bench.py --config 5 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/r5v_c5prof.json 2> gpurun_out/r5v_c5prof.err
grep -o '"value": [0-9.]*' gpurun_out/r5v_c5prof.json
timeout -k 10 300 python bench.py --config 5 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/r5v_c5q.json 2> gpurun_out/r5v_c5q.err
grep -o '"value": [0-9.]*' gpurun_out/r5v_c5q.json
