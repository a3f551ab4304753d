#!/bin/bash
# HBM traffic and SQ activity of the wavefront kernels from rocprofv3 PMC counters, in separate
# passes (FETCH_SIZE and WRITE_SIZE cannot share a gfx950 TCC pass; no trace domains with --pmc).
#   bash tools/pmc_traffic.sh TAG [STEPS] [CONFIG] [EXTRA]  -> gpurun_out/pmc_TAG_*/ + gpurun_out/pmc_TAG.json
# (EXTRA: further bench.py arguments, e.g. "--t8 1" for config 5 with Transform8x8Mode 1)
# The run is the bench's pipelined stream of BASELINE config CONFIG (2, 3 or 5): one IDR picture +
# (pipeline fill + STEPS) P pictures, drained at the end (bench.py completes every picture in flight
# before it exits); tools/pmc_parse.py reads the fill from the pass's bench line.
TAG=${1:-r1}
STEPS=${2:-30}
CONFIG=${3:-2}
EXTRA=${4:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
  name=$(echo "$c" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 600 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_${TAG}_${name}" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --config "$CONFIG" --steps "$STEPS" --warmup 0 --no-cpu-baseline --no-host-path $EXTRA \
      > "gpurun_out/pmc_${TAG}_${name}.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_parse.py "$TAG" "$CONFIG" > "gpurun_out/pmc_${TAG}.json" && cat "gpurun_out/pmc_${TAG}.json"
