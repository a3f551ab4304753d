#!/bin/bash
# GPU session script: parity tests, then (only if no crash) a short bench.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" -p no:cacheprovider > gpurun_out/r1_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/r1_pytest.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r1_bench.log 2>&1
  echo "bench rc=$?"
  tail -5 gpurun_out/r1_bench.log
fi
