#!/bin/bash
# Dynamic VALU / LDS instruction split of k_mb_analyse (config 2): PMC counts of variants built
# with parts removed (-DJMH_EXP bits: 1 no sub-pel SATD, 2 no Intra4x4 slots, 4 no SAD strips);
# the results of those variants are wrong on purpose -- only the instruction counts are read.
#   CPU side: bash tools/valu_split.sh build      GPU side: bash tools/valu_split.sh run TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R/h264-jm-commentary_amd/csrc" || exit 1
if [ "$1" = build ]; then
    for e in 1 2 4 7; do
        /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DJMH_EXP=$e -shared jmh_kernels.hip jmh_analyse.hip \
            jmh_fullsearch.hip jmh_epzs.hip jmh_intra8.hip jmh_final.hip jmh_block.hip jmh_hbd.hip jmhip_abi.hip -o /tmp/libjmhip_exp$e.so || exit 1
        mkdir -p "$R/tools/exp" && cp /tmp/libjmhip_exp$e.so "$R/tools/exp/"
    done
    exit 0
fi
TAG=${2:-exp}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
cp h264-jm-commentary_amd/csrc/libjmhip.so /tmp/libjmhip_base.so
for e in 0 1 2 4 7; do
    if [ $e = 0 ]; then cp /tmp/libjmhip_base.so h264-jm-commentary_amd/csrc/libjmhip.so
    else cp tools/exp/libjmhip_exp$e.so h264-jm-commentary_amd/csrc/libjmhip.so; fi
    timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d "$R/gpurun_out/${TAG}_$e" -o pmc --output-format csv -- \
        python3 "$R/bench.py" --steps 20 --warmup 0 --no-cpu-baseline --no-host-path > "gpurun_out/${TAG}_$e.log" 2>&1
    rc=$?; echo "variant $e rc=$rc"
    [ $rc -eq 0 ] || { cp /tmp/libjmhip_base.so h264-jm-commentary_amd/csrc/libjmhip.so; exit $rc; }
done
cp /tmp/libjmhip_base.so h264-jm-commentary_amd/csrc/libjmhip.so
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
for e in (0, 1, 2, 4, 7):
    tot = collections.Counter(); n = collections.Counter()
    for f in glob.glob(f"gpurun_out/{tag}_{e}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("k_mb_analyse"):
                tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(e, {k: round(v / max(1, n[k])) for k, v in tot.items()})
PY
