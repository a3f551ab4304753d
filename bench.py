#!/usr/bin/env python3
"""bench.py — JM hot path on MI355X: ME + transform megapixels/s, 1080p FFS SR=32.

One step = one P picture of the hot path with inputs resident in HBM, referencing the previous
picture's deblocked reconstruction: the whole macroblock wavefront (k_mb_analyse: FFS SAD table
+ argmin, sub-pel SATD search on the fly from the reference, intra decisions; k_mb_final: RDO-off
mode decision, luma/chroma TQ + reconstruction, deblocking) over all 8160 macroblocks of a coded
1920x1088 picture.  Pictures are pipelined: picture q runs diagonal d once picture q-1 has
finished diagonal d + PIPE_LAG, so ~15 pictures share each launch; the timed region holds the
pipeline fill and drain (sync on both sides).  Entropy coding is excluded, as in JM's
ME/transform time.  Multi-GPU: one independent stream per rank (seed = rank), no
collective in the data path; a gloo barrier brackets the timed region and the maximum time over
ranks is used (h264-jm-commentary_amd/streams.py).

--config 3 runs BASELINE.json's config 3 instead (a variant line, not the headline metric):
2160p synthetic, High profile, EPZS (SearchMode 3) + adaptive 8x8 transform (Transform8x8Mode 1).

Prints ONE JSON line (rank 0).
"""
import argparse
import importlib.util
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "h264-jm-commentary_amd")

METRIC = "ME+transform megapixels/sec @1080p FullSearch SR=32; bit-exact bitstream vs JM"
# BASELINE.json configs measured here: 2 (the headline) and 3 (variant)
CONFIGS = {
    2: dict(metric=METRIC, disp=(1920, 1080), coded=(1920, 1088), search_mode=0, t8=0,
            workload="1080p synthetic YUV420 (coded 1920x1088), Baseline, {sm} SearchRange=32, RestrictSearchRange=2, "
                     "UseHadamard=1, 7 inter block sizes, RDO off, QP 28, P pictures (one independent stream per GPU)"),
    3: dict(metric="ME+transform megapixels/sec @2160p High EPZS SR=32 + 8x8 transform (config 3)", disp=(3840, 2160),
            coded=(3840, 2160), search_mode=3, t8=1,
            workload="2160p synthetic YUV420, High profile (ProfileIDC 100), EPZS SearchMode=3 SearchRange=32, "
                     "Transform8x8Mode=1 (Intra8x8 + TransformDecision), UseHadamard=1, 7 inter block sizes, RDO off, "
                     "QP 28, P pictures (one independent stream per GPU)"),
}
DISP_W, DISP_H = 1920, 1080
W, H = 1920, 1088
SR, QP = 32, 28
NMB = (W // 16) * (H // 16)
# algorithmic HBM bytes per coded picture: current 1.5 B/px + reference 1.5 B/px
# (each read once) + reconstruction 1.5 B/px and deblocked reconstruction 1.5 B/px written +
# levels (int16 per sample) 3.0 B/px, plus per-MB side data (MVs, refs, modes, cbp) 80 B/MB
BYTES_PER_PIXEL = 9.0
SIDE_BYTES_PER_MB = 80
BYTES_PER_FRAME = W * H * BYTES_PER_PIXEL + NMB * SIDE_BYTES_PER_MB
HBM_PEAK_GBS = 8000.0                                    # MI355X_MICROARCH.md (spec)
# integer search absolute differences per picture (FFS SAD table) and the v_sad_u8 peak:
# 4 absolute differences per lane-op, 256 CU x 64 lanes/clk x 2.4 GHz
AD_PER_FRAME = NMB * (2 * SR + 1) ** 2 * 256
VALU_SAD_PEAK_TADS = 256 * 64 * 4 * 2.4e9 / 1e12


def load_module(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def use_config(k):
    """switch the module-level workload constants to BASELINE.json config k"""
    global DISP_W, DISP_H, W, H, NMB, BYTES_PER_FRAME, AD_PER_FRAME
    c = CONFIGS[k]
    (DISP_W, DISP_H), (W, H) = c["disp"], c["coded"]
    NMB = (W // 16) * (H // 16)
    BYTES_PER_FRAME = W * H * BYTES_PER_PIXEL + NMB * SIDE_BYTES_PER_MB
    AD_PER_FRAME = NMB * (2 * SR + 1) ** 2 * 256
    return c


def cpu_one_picture(seed, search_mode, t8=0):
    """Seconds the oracle (JM restated in C, scalar -O2, one thread) takes for one P picture of the
    configured size on stream `seed` (UnifiedOneForthPix + encode_one_macroblock per MB).  Runs in a child
    process (bench.py --cpu-worker): no GPU is touched."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    jm = load_module("jmhip", os.path.join(PKG, "jmhip.py"))
    frames = [jm.synth_frame(DISP_W, DISP_H, seed, i) for i in range(2)]
    o = oracle_lib.OracleEncoder(W, H, search_range=SR, search_mode=search_mode, transform_8x8_mode=t8)
    _, rec = o.encode(*frames[0], jm.JMH_I_SLICE, QP)
    t0 = time.perf_counter()
    o.set_reference(*rec)
    o.encode(*frames[1], jm.JMH_P_SLICE, QP)
    dt = time.perf_counter() - t0
    o.close()
    return dt


def cpu_workers(n, config, search_mode):
    """n concurrent child processes (distinct seeds); their per-picture seconds."""
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", str(k), str(config), str(search_mode)],
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True) for k in range(n)]
    return [float(p.communicate()[0].split()[-1]) for p in procs]


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(config=2, search_mode=0):
    """The CPU path timed on this node's host cores: one process on one core (JM is
    single threaded; the reported baseline), and n processes on distinct streams at once
    (aggregate, n = min(16, cores available to this process))."""
    one = cpu_workers(1, config, search_mode)[0]
    n = max(1, min(16, len(os.sched_getaffinity(0))))
    many = cpu_workers(n, config, search_mode)
    mode = {0: "FFS", -1: "full search", 3: "EPZS"}[search_mode] + (" + 8x8 transform" if CONFIGS[config]["t8"] else "")
    return {"value": round(DISP_W * DISP_H / 1e6 / one, 4), "unit": "MP/s", "cores": 1, "kind": "port",
            "sample": f"one {DISP_W}x{DISP_H} P picture (coded {W}x{H}, {NMB} MBs, {mode} SR=32, QP {QP}) incl. "
                      f"quarter-pel interpolation, oracle/liboracle.so -O2 scalar, {one:.1f} s, on {cpu_model()}",
            "all_cores": {"value": round(n * DISP_W * DISP_H / 1e6 / max(many), 4), "unit": "MP/s", "cores": n,
                          "sample": f"{n} processes, one P picture each on distinct streams, concurrently, "
                                    f"{max(many):.1f} s wall"}}


def read_pmc_traffic():
    """HBM bytes per macroblock of k_mb_analyse measured by rocprofv3 PMC passes
    (tools/pmc_traffic.sh -> profiles/pmc_traffic.json), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            return json.load(f)["kernels"]["k_mb_analyse"]["hbm_bytes_per_mb"]
    except (OSError, ValueError, KeyError, TypeError):
        return None


def main():
    if len(sys.argv) == 5 and sys.argv[1] == "--cpu-worker":    # child of cpu_baseline()
        c = use_config(int(sys.argv[3]))
        print(cpu_one_picture(int(sys.argv[2]), int(sys.argv[4]), c["t8"]), flush=True)
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", type=int, default=2, choices=(2, 3),
                    help="BASELINE.json config: 2 = 1080p Baseline FFS (the headline), 3 = 2160p High EPZS + 8x8")
    ap.add_argument("--search-mode", type=int, default=None, choices=(0, -1, 3),
                    help="override the config's SearchMode (config 2 variants: -1 full search, 3 EPZS)")
    args = ap.parse_args()
    cfg = use_config(args.config)
    search_mode = cfg["search_mode"] if args.search_mode is None else args.search_mode

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")

    jm = load_module("jmhip", os.path.join(PKG, "jmhip.py"))
    streams = load_module("jmh_streams", os.path.join(PKG, "streams.py"))
    frames = [jm.synth_frame(DISP_W, DISP_H, rank, i) for i in range(3)]
    enc = jm.Encoder(W, H, device=local, search_range=SR, search_mode=search_mode, slots=3, kernel_timing=True,
                     transform_8x8_mode=cfg["t8"])
    stream = streams.PStream(enc, frames, QP)
    dt = streams.timed_run(stream, args.steps, args.warmup, dist, on_start=enc.timing)   # on_start resets the event sums
    tm = enc.timing()                                     # event sums of the timed steps only

    if rank != 0:
        if dist is not None:
            dist.barrier()
        enc.close()
        return
    value = world * args.steps * DISP_W * DISP_H / 1e6 / dt
    pictures = max(1, tm.pictures)
    an_launch_ms = tm.analyse_ms / max(1, tm.analyse_launches)
    an_per_pic = tm.ticks / pictures                     # one k_mb_analyse + one k_mb_final per tick
    mbs_per_launch = tm.tick_mbs / max(1, tm.ticks)      # MBs of all pictures in flight, per tick
    bytes_per_launch = BYTES_PER_FRAME / NMB * mbs_per_launch
    achieved_gbs = bytes_per_launch / (an_launch_ms * 1e-3) / 1e9
    mb_ms_pic = tm.mb_ms / pictures
    pmc = read_pmc_traffic() if args.config == 2 and search_mode == 0 else None   # PMC pass is for config 2
    sm_name = {0: "FFS SearchMode=0", -1: "full search SearchMode=-1", 3: "EPZS SearchMode=3"}[search_mode]
    out = {
        "metric": cfg["metric"],
        "value": round(value, 3),
        "unit": "MP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": cfg["workload"].replace("{sm}", sm_name),
            "global_batch": world,
            "parallelism": f"streams{world}",
            "pipeline_depth": enc.depth,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved_gbs, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 6),
            "traffic": round(pmc * mbs_per_launch) if pmc else None,
            "kernel": "k_mb_analyse" if search_mode == 0 else
                      "k_mb_me_full + k_mb_analyse" + (" + k_mb_intra8" if cfg["t8"] else "") + " (the tick's analysis launches)",
            "algorithmic_bytes_per_launch": round(bytes_per_launch),
            "avg_launch_ms": round(an_launch_ms, 5),
            "launches_per_picture": round(an_per_pic, 2),
            "mbs_per_launch": round(mbs_per_launch, 1),
        },
        "valu_roofline": None if search_mode != 0 else {
            "note": "integer-search absolute differences (v_sad_u8) over the wavefront time",
            "achieved": round(AD_PER_FRAME / (mb_ms_pic * 1e-3) / 1e12, 4),
            "peak": round(VALU_SAD_PEAK_TADS, 2),
            "unit": "T abs-diff/s",
            "frac": round(AD_PER_FRAME / (mb_ms_pic * 1e-3) / 1e12 / VALU_SAD_PEAK_TADS, 6),
        },
        # per-launch averages (sampled every 8th diagonal) x launches per picture
        "kernel_ms_per_picture": {"wavefront": round(mb_ms_pic, 4),
                                  "k_mb_analyse": round(an_launch_ms * an_per_pic, 4),
                                  "k_mb_final": round(tm.final_ms / max(1, tm.final_launches) * an_per_pic, 4),
                                  "k_interp": round(tm.interp_ms / max(1, tm.interps), 4)},
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.config, search_mode)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
    enc.close()


if __name__ == "__main__":
    main()
