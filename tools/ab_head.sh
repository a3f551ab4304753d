#!/bin/bash
# Build the committed HEAD's libjmhip.so as an A/B variant: csrc/ab/libjmhip_head.so
# (git archive of HEAD's csrc + include into a temp dir, compiled like tools/fastbuild.sh)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive HEAD h264-jm-commentary_amd/csrc include | tar -x -C "$T"
cd "$T/h264-jm-commentary_amd/csrc"
pids=()
for f in jmh_kernels jmh_analyse jmh_flow jmh_fullsearch jmh_epzs jmh_intra8 jmh_final jmh_block jmh_hbd jmh_rdo jmhip_abi; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -c $f.hip -o "$T/$f.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
mkdir -p "$R/h264-jm-commentary_amd/csrc/ab"
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared "$T"/*.o -o "$R/h264-jm-commentary_amd/csrc/ab/libjmhip_head.so"
rm -rf "$T"
echo "built ab/libjmhip_head.so from $(git -C "$R" rev-parse --short HEAD)"
