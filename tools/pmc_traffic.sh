#!/bin/bash
# HBM traffic of the wavefront kernels from rocprofv3 PMC counters, one counter per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a gfx950 TCC pass), then SQ occupancy/stall counters.
#   bash tools/pmc_traffic.sh TAG      -> gpurun_out/pmc_TAG_{fetch,write,sq}/ + gpurun_out/pmc_TAG.json
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"; do
  name=$(echo "$c" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 600 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_${TAG}_${name}" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "gpurun_out/pmc_${TAG}_${name}.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_parse.py "$TAG" > "gpurun_out/pmc_${TAG}.json" && cat "gpurun_out/pmc_${TAG}.json"
