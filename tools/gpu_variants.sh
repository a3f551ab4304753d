#!/bin/bash
# Variant benches on one GPU: config 2 (regression check), config 3 (2160p High EPZS + 8x8, with
# the CPU baseline), config 2 with EPZS, and a rocprofv3 kernel-stats pass over config 3.
#   bash tools/gpu_variants.sh TAG
TAG=${1:-var}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_c2.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_c2.log | cut -c1-200
timeout -k 10 400 python bench.py --config 3 --steps 80 --warmup 24 > gpurun_out/${TAG}_c3.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_c3.log
timeout -k 10 300 python bench.py --search-mode 3 --no-cpu-baseline > gpurun_out/${TAG}_c2epzs.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_c2epzs.log | cut -c1-200
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}" -o ${TAG} --output-format csv -- python3 "$R/bench.py" --config 3 --steps 80 --warmup 24 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
find gpurun_out/prof_${TAG} -name "*kernel_stats*" -exec cat {} \;
exit $rc
