T=$1
timeout -k 10 400 python -u -m pytest tests/test_rdo_gpu.py -k ffs -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${T}_ffs.log 2>&1; tail -2 gpurun_out/${T}_ffs.log
bash tools/gpu_session.sh $T c5ffs > /dev/null || exit 1
grep -o '"value": [0-9.]*' gpurun_out/${T}_c5ffs_bench.json
JMH_PHASE_PROF=16020 timeout -k 10 300 python bench.py --config 5 --search-mode 0 --steps 20 --no-cpu-baseline --no-host-path > gpurun_out/${T}_phase.json 2> gpurun_out/${T}_phase.err
grep jmh_phase gpurun_out/${T}_phase.err | tail -1
