#!/bin/bash
# Where the waves of the config-2 tick wait: two SQ passes over the bench's
# pipelined stream (separate runs, no trace domains with --pmc), summarised per kernel by
# tools/pmc_wait.py: WAIT_ANY / WAIT_INST_ANY / ACTIVE split of SQ_WAVE_CYCLES, and the mean
# latency (Little's law: SQ_INST_LEVEL_x / SQ_INSTS_x) and in-flight share of VMEM, LDS and SMEM.
#   bash tools/pmc_wait.sh TAG [STEPS] -> gpurun_out/pmcw_TAG_{a,b}/ + gpurun_out/pmcw_TAG.json
TAG=${1:-r1}
STEPS=${2:-30}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS" \
         "SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAVES"; do
  p=$([ $i -eq 0 ] && echo a || echo b); i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $c -d "$R/gpurun_out/pmcw_${TAG}_$p" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --steps "$STEPS" --warmup 0 --no-cpu-baseline --no-host-path > "gpurun_out/pmcw_${TAG}_$p.log" 2>&1
  rc=$?; echo "pmc pass $p rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_wait.py "$TAG" > "gpurun_out/pmcw_${TAG}.json" && cat "gpurun_out/pmcw_${TAG}.json"
