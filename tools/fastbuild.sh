#!/bin/bash
# Development build of libjmhip.so: one object per translation unit (rebuilt only when its source
# or a header is newer), compiled in parallel, then linked.  OUT=path overrides the library,
# DEFS="-D..." adds defines (A/B variants use their own object directory).
set -e
cd "$(dirname "$0")/../h264-jm-commentary_amd/csrc"
DEFS=${DEFS:-}
OUT=${OUT:-libjmhip.so}
OBJ=.obj/$(echo "$DEFS" | tr -c 'A-Za-z0-9_=\n' '_' )
mkdir -p "$OBJ"
HDRS="jmh_device.h jmh_common.h jmh_epzs.h jmh_intra.h jmh_i4.h jmh_deblock.h jmh_intra8.h jmh_cabac_rate.h jmh_cavlc_rate.h jmh_final.h jmh_cabac_tables.h ../../include/jmhip.h"
pids=()
for f in jmh_kernels jmh_analyse jmh_flow jmh_fullsearch jmh_epzs jmh_intra8 jmh_final jmh_block jmh_hbd jmh_rdo jmhip_abi; do
  o=$OBJ/$f.o
  extra=""; [ $f = jmh_flow ] && extra=jmh_analyse.hip   # jmh_flow.hip includes jmh_analyse.hip
  if [ ! -f $o ] || [ -n "$(find $f.hip $extra $HDRS -newer $o 2>/dev/null)" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $DEFS -c $f.hip -o $o &
    pids+=($!)
  fi
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared $OBJ/*.o -o "$OUT"
echo "built $OUT"
