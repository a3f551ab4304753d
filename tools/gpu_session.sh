#!/bin/bash
# One GPU session on the gpurun box, as a list of named steps (each under its own time limit;
# the first failing step ends the session):
#   bash tools/gpu_session.sh TAG step [step ...]
# steps:
#   build   make the product + oracle in-tree (normally done here on the CPU beforehand)
#   peak    tools/sad_peak_bin                       -> gpurun_out/TAG_sad_peak.json
#   tests   pytest -m gpu (all)                      -> gpurun_out/TAG_pytest.log
#   fast    pytest -m "gpu and not slow"             -> gpurun_out/TAG_pytest.log
#   rdo     pytest tests/test_rdo_gpu.py (RDOptimization 1; failures reported, not fatal)
#   smoke   __graft_entry__.smoke()                  -> gpurun_out/TAG_smoke.log
#   bench   bench.py (defaults, with CPU baseline)   -> gpurun_out/TAG_bench.json
#   bench20 bench.py --steps 20 --warmup 5 (the driver's invocation, no CPU baseline)
#   benchf8 bench20 with JMH_FINAL_OCC8=1 (k_mb_final's 8-per-CU build for every tick: A/B)
#   c3      bench.py --config 3 (with CPU baseline)  -> gpurun_out/TAG_c3_bench.json
#   c3s     config 3 with SliceMode 1, SliceArgument 240 (config 5's one-row slices, 8-bit, CAVLC)
#   c5      bench.py --config 5 (High 10, RDO on, 240-MB slices; with CPU baseline)
#   c5q     the same, 60 steps, no CPU baseline / host path (a quick GPU number)
#   c5off   config 5's RDO-off variant (EPZS + 8x8 transform)
#   c5t8    config 5 with Transform8x8Mode 1 (RDO on: 8x8-transform candidates, I8MB; with CPU baseline)
#   lencodc5 lencodc3 with one slice and with SliceArgument 240 (135 one-row slices per picture)
#   prof    rocprofv3 --kernel-trace --stats of the bench -> gpurun_out/prof_TAG/
#   profc3  the same for config 3
#   pmc     tools/pmc_traffic.sh (HBM bytes + SQ counters, separate passes), config 2
#   pmc3 / pmc5  the same for config 3 / config 5 (RDO on); pmc5t8 config 5 with Transform8x8Mode 1
#   lencod  the product lencod end to end on an I420 file (tools/make_yuv.py), 1080p, 60 pictures
#           (FFS SR 32), WriterThreads 0 / 4 / 8 -> gpurun_out/TAG_lencod1080_w*.log
#   lencodc3 the same for the config-3 shape (2160p High, EPZS + 8x8), 30 pictures, 8 writers
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name limit cmd...
    local name=$1 lim=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$lim" "$@"
    local rc=$?
    echo "== $name rc=$rc"
    return $rc
}
for s in "$@"; do
  case $s in
    build)  run build 600 make -s -j16 all || exit $? ;;
    peak)   run peak 120 tools/sad_peak_bin > gpurun_out/${TAG}_sad_peak.json || exit $?
            cat gpurun_out/${TAG}_sad_peak.json ;;
    tests)  run tests 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
                > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc ;;
    hbd)    run hbd 600 python -u -m pytest tests -v -m gpu -k "high10 or lencod_bitstream" -p no:cacheprovider --timeout 300 \
                --timeout-method thread > gpurun_out/${TAG}_hbd.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_hbd.log
            [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    rdo)    run rdo 900 python -u -m pytest tests/test_rdo_gpu.py -v -p no:cacheprovider --timeout 300 --timeout-method thread \
                > gpurun_out/${TAG}_rdo.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_rdo.log
            [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    fast)   run fast 600 python -u -m pytest tests -x -v -m "gpu and not slow" -p no:cacheprovider --timeout 120 \
                --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_pytest.log
            [ $rc -eq 0 ] || exit $rc ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
            cat gpurun_out/${TAG}_smoke.log ;;
    bench)  run bench 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
            cat gpurun_out/${TAG}_bench.json ;;
    bench20) run bench20 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench20.json || exit $?
            cat gpurun_out/${TAG}_bench20.json ;;
    benchf8) JMH_FINAL_OCC8=1 run benchf8 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_benchf8.json || exit $?
            cat gpurun_out/${TAG}_benchf8.json ;;
    c3)     run c3 900 python bench.py --config 3 > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3_bench.err || exit $?
            cat gpurun_out/${TAG}_c3_bench.json ;;
    c5)     run c5 1100 python bench.py --config 5 > gpurun_out/${TAG}_c5_bench.json 2> gpurun_out/${TAG}_c5_bench.err || exit $?
            cat gpurun_out/${TAG}_c5_bench.json ;;
    c5t8)   run c5t8 1100 python bench.py --config 5 --t8 1 > gpurun_out/${TAG}_c5t8_bench.json 2> gpurun_out/${TAG}_c5t8_bench.err || exit $?
            cat gpurun_out/${TAG}_c5t8_bench.json ;;
    c5q)    run c5q 600 python bench.py --config 5 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_c5q_bench.json \
                2> gpurun_out/${TAG}_c5q_bench.err || exit $?
            cat gpurun_out/${TAG}_c5q_bench.json ;;
    c5off)  run c5off 900 python bench.py --config 5 --rdo 0 --no-cpu-baseline > gpurun_out/${TAG}_c5off_bench.json \
                2> gpurun_out/${TAG}_c5off_bench.err || exit $?
            cat gpurun_out/${TAG}_c5off_bench.json ;;
    c3s)    run c3s 900 python bench.py --config 3 --slice-mbs 240 > gpurun_out/${TAG}_c3s_bench.json 2> gpurun_out/${TAG}_c3s_bench.err || exit $?
            cat gpurun_out/${TAG}_c3s_bench.json ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}" -o ${TAG} --output-format csv -- \
                python3 "$R/bench.py" --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
            find gpurun_out/prof_${TAG} -name "*kernel_stats*" -exec cat {} \; ;;
    profc5) run profc5 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_c5" -o ${TAG}_c5 --output-format csv -- \
                python3 "$R/bench.py" --config 5 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_profc5.log 2>&1 || exit $?
            find gpurun_out/prof_${TAG}_c5 -name "*kernel_stats*" -exec cat {} \; ;;
    profc5t8) run profc5t8 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_c5t8" -o ${TAG}_c5t8 --output-format csv -- \
                python3 "$R/bench.py" --config 5 --t8 1 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_profc5t8.log 2>&1 || exit $?
            find gpurun_out/prof_${TAG}_c5t8 -name "*kernel_stats*" -exec cat {} \; ;;
    profc3) run profc3 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_c3" -o ${TAG}_c3 --output-format csv -- \
                python3 "$R/bench.py" --config 3 --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_profc3.log 2>&1 || exit $?
            find gpurun_out/prof_${TAG}_c3 -name "*kernel_stats*" -exec cat {} \; ;;
    lencod) run mkyuv 300 python tools/make_yuv.py /tmp/s1080.yuv 1920 1080 60 || exit $?
            for wt in 0 4 8; do
              run lencod_w$wt 600 h264-jm-commentary_amd/host/build/lencod -p InputFile=/tmp/s1080.yuv -p FramesToBeEncoded=60 \
                -p SourceWidth=1920 -p SourceHeight=1080 -p SearchRange=32 -p WriterThreads=$wt -p OutputFile=/tmp/l1080_$wt.264 \
                > gpurun_out/${TAG}_lencod1080_w$wt.log 2>&1 || exit $?
              tail -5 gpurun_out/${TAG}_lencod1080_w$wt.log
            done
            cmp /tmp/l1080_0.264 /tmp/l1080_4.264 && cmp /tmp/l1080_0.264 /tmp/l1080_8.264 && echo "bitstreams identical" || exit 1 ;;
    lencodc3) run mkyuv 300 python tools/make_yuv.py /tmp/s2160.yuv 3840 2160 30 || exit $?
            run lencodc3 900 h264-jm-commentary_amd/host/build/lencod -p InputFile=/tmp/s2160.yuv -p FramesToBeEncoded=30 \
                -p SourceWidth=3840 -p SourceHeight=2160 -p SearchRange=32 -p ProfileIDC=100 -p Transform8x8Mode=1 \
                -p SearchMode=3 -p WriterThreads=8 -p OutputFile=/tmp/l2160.264 > gpurun_out/${TAG}_lencod2160.log 2>&1 || exit $?
            tail -5 gpurun_out/${TAG}_lencod2160.log ;;
    lencodc5) run mkyuv 300 python tools/make_yuv.py /tmp/s2160.yuv 3840 2160 30 || exit $?
            for sl in 0 240; do
              run lencodc5_$sl 900 h264-jm-commentary_amd/host/build/lencod -p InputFile=/tmp/s2160.yuv -p FramesToBeEncoded=30 \
                -p SourceWidth=3840 -p SourceHeight=2160 -p SearchRange=32 -p ProfileIDC=100 -p Transform8x8Mode=1 \
                -p SearchMode=3 -p WriterThreads=8 -p SliceMode=$((sl > 0)) -p SliceArgument=$((sl > 0 ? sl : 50)) \
                -p OutputFile=/tmp/l2160_$sl.264 > gpurun_out/${TAG}_lencod2160_slices$sl.log 2>&1 || exit $?
              tail -3 gpurun_out/${TAG}_lencod2160_slices$sl.log
            done ;;
    pmc)    run pmc 900 bash tools/pmc_traffic.sh "$TAG" || exit $? ;;
    pmc3)   run pmc3 900 bash tools/pmc_traffic.sh "${TAG}_c3" 30 3 || exit $? ;;
    pmc5)   run pmc5 900 bash tools/pmc_traffic.sh "${TAG}_c5" 30 5 || exit $? ;;
    pmc5t8) run pmc5t8 900 bash tools/pmc_traffic.sh "${TAG}_c5t8" 30 5 "--t8 1" || exit $? ;;
    pmc5ffs) run pmc5ffs 900 bash tools/pmc_traffic.sh "${TAG}_c5ffs" 30 5 "--search-mode 0" || exit $? ;;
    proft)  JMH_FLOW=0 run proft 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_tick" -o ${TAG}_tick --output-format csv -- \
                python3 "$R/bench.py" --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_proft.log 2>&1 || exit $?
            find gpurun_out/prof_${TAG}_tick -name "*kernel_stats*" -exec cat {} \; ;;
    c5ffs)  run c5ffs 900 python bench.py --config 5 --search-mode 0 --steps 60 --no-cpu-baseline --no-host-path > gpurun_out/${TAG}_c5ffs_bench.json \
                2> gpurun_out/${TAG}_c5ffs_bench.err || exit $?
            cat gpurun_out/${TAG}_c5ffs_bench.json ;;
    *)      echo "unknown step $s"; exit 2 ;;
  esac
done
