#!/usr/bin/env python3
"""bench.py — JM hot path on MI355X: ME + transform megapixels/s, 1080p FFS SR=32.

One step = one P picture of the hot path with inputs resident in HBM: quarter-pel
interpolation of the new reference (the previous picture's reconstruction) + the full
macroblock wavefront (integer FFS SAD table + argmin, sub-pel SATD search, RDO-off mode
decision incl. intra, luma/chroma TQ + reconstruction) for all 8160 macroblocks of a coded
1920x1088 picture.  Entropy coding and deblocking are excluded, as JM's MET column is
(BASELINE.md).  Multi-GPU: one independent stream per rank (seed = rank), no collective in the
data path; a gloo barrier brackets the timed region and the max time over ranks is used.

Prints ONE JSON line (rank 0).
"""
import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "h264-jm-commentary_amd")

METRIC = "ME+transform megapixels/sec @1080p FullSearch SR=32; bit-exact bitstream vs JM"
DISP_W, DISP_H = 1920, 1080
W, H = 1920, 1088
SR, QP = 32, 28
NMB = (W // 16) * (H // 16)
# algorithmic work per coded picture
AD_PER_FRAME = NMB * (2 * SR + 1) ** 2 * 256          # integer-search absolute differences
BYTES_PER_PIXEL = 7.5                                    # cur 1.5 + ref 1.5 + recon 1.5 + levels 3.0
SIDE_BYTES_PER_MB = 80
BYTES_PER_FRAME = W * H * BYTES_PER_PIXEL + NMB * SIDE_BYTES_PER_MB
HBM_PEAK_GBS = 8000.0                                    # MI355X_MICROARCH.md (spec)
# v_sad_u8: 4 absolute differences per lane-op; 256 CU x 128 lanes/clk x 2.4 GHz (nominal)
VALU_SAD_PEAK_TADS = 256 * 128 * 4 * 2.4e9 / 1e12


def load_pkg():
    spec = importlib.util.spec_from_file_location("jmhip", os.path.join(PKG, "jmhip.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["jmhip"] = mod
    spec.loader.exec_module(mod)
    return mod


def cpu_baseline(jm, frames):
    """The oracle (JM restated in C, scalar -O2, 1 thread) on one full 1080p P picture."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    o = oracle_lib.OracleEncoder(W, H, search_range=SR)
    _, rec = o.encode(*frames[0], jm.JMH_I_SLICE, QP)
    t0 = time.perf_counter()
    o.set_reference(*rec)                                 # UnifiedOneForthPix
    o.encode(*frames[1], jm.JMH_P_SLICE, QP)              # encode_one_macroblock x 8160
    dt = time.perf_counter() - t0
    o.close()
    return {"value": round(DISP_W * DISP_H / 1e6 / dt, 4), "unit": "MP/s", "cores": 1, "kind": "port",
            "sample": f"one 1920x1080 P picture (coded 1920x1088, 8160 MBs, FFS SR=32, QP {QP}) incl. "
                      f"quarter-pel interpolation, oracle/liboracle.so -O2 scalar, {dt:.1f} s"}


def read_pmc_traffic():
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")

    jm = load_pkg()
    frames = [jm.synth_frame(DISP_W, DISP_H, rank, i) for i in range(3)]
    enc = jm.Encoder(W, H, device=local, search_range=SR, slots=3)
    for i, f in enumerate(frames):
        enc.load_frame(i, *f)
    enc.encode_slot(0, jm.JMH_I_SLICE, QP)                # IDR picture -> first reference
    enc.sync()

    def step(i):
        enc.set_reference_slot(-1)                        # previous recon -> quarter-pel planes
        enc.encode_slot(1 + (i % 2), jm.JMH_P_SLICE, QP)  # P picture: the whole MB wavefront

    for i in range(args.warmup):
        step(i)
    enc.sync()
    enc.timing()                                          # reset the event sums

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    enc.sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    enc.sync()
    t1 = time.perf_counter()
    barrier()
    dt = t1 - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    tm = enc.timing()

    if rank != 0:
        if dist is not None:
            dist.barrier()
        return
    value = world * args.steps * DISP_W * DISP_H / 1e6 / dt
    ms_per_step = dt * 1e3 / args.steps
    launches = max(1, tm.mb_launches)
    mb_ms_pic = tm.mb_ms / max(1, tm.pictures)
    avg_launch_ms = mb_ms_pic / launches
    achieved_gbs = (BYTES_PER_FRAME / launches) / (avg_launch_ms * 1e-3) / 1e9
    pmc = read_pmc_traffic()
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "MP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": "1080p synthetic YUV420 (coded 1920x1088), Baseline, FFS SearchMode=0 "
                        "SearchRange=32, RestrictSearchRange=2, UseHadamard=1, 7 inter block sizes, "
                        "RDO off, QP 28, P pictures (one independent stream per GPU)",
            "global_batch": world,
            "parallelism": f"streams{world}",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved_gbs, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 6),
            "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
            "kernel": "k_mb_encode",
            "algorithmic_bytes_per_launch": round(BYTES_PER_FRAME / launches),
            "avg_launch_ms": round(avg_launch_ms, 5),
            "launches_per_picture": launches,
        },
        "valu_roofline": {
            "note": "binding roofline: integer-search absolute differences on v_sad_u8",
            "achieved": round(AD_PER_FRAME / (mb_ms_pic * 1e-3) / 1e12, 4),
            "peak": round(VALU_SAD_PEAK_TADS, 2),
            "unit": "T abs-diff/s",
            "frac": round(AD_PER_FRAME / (mb_ms_pic * 1e-3) / 1e12 / VALU_SAD_PEAK_TADS, 6),
        },
        "kernel_ms_per_picture": {"k_mb_encode_wavefront": round(mb_ms_pic, 4),
                                  "k_interp": round(tm.interp_ms / max(1, tm.interps), 4)},
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(jm, frames)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
    enc.close()


if __name__ == "__main__":
    main()
