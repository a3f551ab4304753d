#!/bin/bash
# Config 2 session: full parity suite, config 2 bench, a block profile of one steady-state tick,
# rocprofv3 kernel stats over config 2.
#   bash tools/gpu_c2.sh TAG
TAG=${1:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-250
JMH_BLOCK_PROF=3001 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/${TAG}_bprof.log 2>&1 || exit $?
grep jmh_blocks gpurun_out/${TAG}_bprof.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}" -o ${TAG} --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
find gpurun_out/prof_${TAG} -name "*kernel_stats*" -exec cat {} \;
exit $rc
