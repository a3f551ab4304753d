#!/bin/bash
# Config 3 session: EPZS / High-profile / pipelined parity subset, config 3 bench (300 pictures),
# rocprofv3 kernel stats over config 3.
#   bash tools/gpu_c3.sh TAG
TAG=${1:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "epzs or high_profile or pipelined or lencod or ipp_configs" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 3 --steps 300 --warmup 40 --no-cpu-baseline > gpurun_out/${TAG}_c3.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_c3.log | cut -c1-300
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}" -o ${TAG} --output-format csv -- python3 "$R/bench.py" --config 3 --steps 300 --warmup 40 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
find gpurun_out/prof_${TAG} -name "*kernel_stats*" -exec cat {} \;
exit $rc
