#!/bin/bash
# One GPU session: parity suite (incl. 1080p), bench (with CPU baseline), rocprofv3 kernel trace.
#   bash tools/gpu_session.sh TAG [pytest-args...]
# Outputs: gpurun_out/TAG_pytest.log, TAG_bench.log, prof_TAG/ (kernel stats csv)
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider "$@" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${TAG}_bench.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}" -o ${TAG} --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"
find gpurun_out/prof_${TAG} -name "*kernel_stats*" -exec cat {} \;
exit $rc
