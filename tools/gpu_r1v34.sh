#!/bin/bash
# One GPU session: full parity suite, config 2 bench (with CPU baseline), config 3 bench, and a
# rocprofv3 kernel-stats pass over config 2.
#   bash tools/gpu_r1v34.sh TAG
TAG=${1:-r1_v34}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
timeout -k 10 300 python bench.py --config 3 --steps 80 --warmup 40 --no-cpu-baseline > gpurun_out/${TAG}_c3.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_c3.log | cut -c1-400
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}" -o ${TAG} --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
find gpurun_out/prof_${TAG} -name "*kernel_stats*" -exec cat {} \;
exit $rc
