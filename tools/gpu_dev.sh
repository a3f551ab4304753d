#!/bin/bash
# Development loop on one GPU: a parity subset (-k EXPR), the phase profile of one MB, a bench.
#   bash tools/gpu_dev.sh TAG "pytest -k expr" "bench args" [SEARCH_MODE]
TAG=${1:-dev}; K=${2:-"epzs or ipp_configs or lencod or pipelined"}; BA=${3:-"--search-mode 3 --no-cpu-baseline"}; SM=${4:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
SEARCH_MODE=$SM JMH_PHASE_PROF=4000 timeout -k 10 120 python tools/phase_prof.py 2>&1 | grep jmh_phase | tail -1 || exit $?
timeout -k 10 300 python bench.py $BA > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-330
