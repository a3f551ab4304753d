#!/bin/bash
# Instruction-cache behaviour of the wavefront kernels (the search kernels are 300-380 KB of code):
# SQC_ICACHE_HITS / MISSES and SQ_IFETCH / SQ_IFETCH_LEVEL with wave cycles, separate passes, for
# config 2 (k_mb_analyse) and config 5 (k_rdo_*) -> gpurun_out/pmci_TAG_{c2,c5}_{a,b}/
#   bash tools/pmc_icache.sh TAG
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in 2 5; do
  steps=$([ $cfg -eq 2 ] && echo 30 || echo 12)
  i=0
  for c in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"; do
    p=$([ $i -eq 0 ] && echo a || echo b); i=$((i + 1))
    timeout -s KILL 300 rocprofv3 --pmc $c -d "$R/gpurun_out/pmci_${TAG}_c${cfg}_$p" -o pmc --output-format csv -- \
        python3 "$R/bench.py" --config $cfg --steps $steps --warmup 0 --no-cpu-baseline --no-host-path > "gpurun_out/pmci_${TAG}_c${cfg}_$p.log" 2>&1
    rc=$?; echo "pmc c$cfg pass $p rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
