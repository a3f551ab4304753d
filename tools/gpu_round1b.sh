#!/bin/bash
# GPU session: full parity suite (incl. 1080p), bench with CPU baseline, rocprofv3 kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/r1b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/r1b_pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r1b_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r1b_bench.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r1" -o r1 --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r1b_prof.log 2>&1
echo "prof rc=$?"
find gpurun_out/prof_r1 -name "*stats*" | head
