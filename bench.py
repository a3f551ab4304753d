#!/usr/bin/env python3
"""bench.py — JM hot path on MI355X: ME + transform megapixels/s, 1080p FFS SR=32.

One step = one P picture of the hot path with inputs resident in HBM, referencing the previous
picture's deblocked reconstruction: the whole macroblock wavefront (k_mb_analyse: FFS SAD table
+ argmin, sub-pel SATD search on the fly from the reference, intra decisions; k_mb_final: RDO-off
mode decision, luma/chroma TQ + reconstruction, deblocking) over all 8160 macroblocks of a coded
1920x1088 picture.  The source is SURVEY.md §8d's synthetic sequence (an IDR picture + --frames P
pictures, resident in HBM, cycled).  Pictures are pipelined: picture q runs diagonal d once
picture q-1 has finished diagonal d + PIPE_LAG, so ~16 pictures share each launch.  The timed
region is steady state: the warmup (at least the pipeline depth) fills the pipeline, a barrier +
wait for every issued launch brackets exactly --steps steps on both sides, and exactly --steps
pictures complete inside it (checked: `pictures_completed`), so the value does not depend on
--steps (h264-jm-commentary_amd/streams.py).  Entropy coding is excluded, as in JM's ME/transform
time.

Also reported (never `value`): the PCIe-inclusive rate of the host-buffer path (jmh_frame_push /
jmh_frame_pop: source H2D, results + reconstruction D2H; SURVEY §8d's submit-to-host-visible
timer), the single-picture latency (push -> results host-visible on an empty pipeline), and a
correctness check — the CPU baseline's I + P pictures encoded on the GPU and compared with the
oracle's results of the same run (`verified`).

Multi-GPU (config 4): one independent stream per rank (seed = rank), no collective in the data
path; a gloo barrier brackets the timed region and the maximum time over ranks is used.
`--gpus N` without a launcher spawns N ranks itself (one process per GPU, rank k on device
k mod the device count); under torchrun WORLD_SIZE must equal --gpus.

--config 3 runs BASELINE.json's config 3 instead (a variant line, not the headline metric):
2160p synthetic, High profile, EPZS (SearchMode 3) + adaptive 8x8 transform (Transform8x8Mode 1).
--config 5 runs config 5 (a variant line): 2160p synthetic 10-bit (High 10, 16-bit samples in HBM),
EPZS, SliceMode 1 with 240-MB slices (one MB row), RDOptimization 1 -- the device RD loop with the
CABAC rate of every candidate (k_rdo_inter + k_rdo_intra + k_rdo_final on the RD stage schedule; the bitstream
itself is written on the host, outside the metric as for every config).  --rdo 0 runs the RDO-off
variant of the same shape (EPZS + 8x8 transform).

Prints ONE JSON line (rank 0).
"""
import argparse
import importlib.util
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "h264-jm-commentary_amd")

# `value` times the device-resident path: inputs already in HBM, no H2D / D2H inside the timed
# region.  SURVEY §8d's submit-to-host-visible timer (incl. PCIe) is host_path.pcie_inclusive_mp_s.
TIMER = "device-resident (inputs in HBM, no H2D/D2H in the timed region)"
METRIC = ("ME+transform megapixels/sec @1080p FullSearch SR=32; bit-exact vs the in-repo JM restatement (oracle); "
          + TIMER)
# BASELINE.json configs measured here: 2 (the headline) and 3 (variant)
CONFIGS = {
    # metric_sm: how the metric names the config's own search (BASELINE.json: "FullSearch" for FFS,
    # JM's exact fast full search), replaced when --search-mode measures another one
    2: dict(metric=METRIC, metric_sm="FullSearch", disp=(1920, 1080), coded=(1920, 1088), search_mode=0, t8=0,
            workload="1080p synthetic YUV420 (coded 1920x1088), Baseline, {sm} SearchRange=32, RestrictSearchRange=2, "
                     "UseHadamard=1, 7 inter block sizes, RDO off, QP 28, IDR + {nf}-picture P sequence cycled "
                     "(one independent stream per GPU)"),
    3: dict(metric="ME+transform megapixels/sec @2160p High EPZS SR=32 + 8x8 transform (config 3); " + TIMER, disp=(3840, 2160),
            coded=(3840, 2160), search_mode=3, t8=1,
            workload="2160p synthetic YUV420, High profile (ProfileIDC 100), {sm} SearchRange=32, "
                     "Transform8x8Mode=1 (Intra8x8 + TransformDecision), UseHadamard=1, 7 inter block sizes, RDO off, "
                     "QP 28, IDR + {nf}-picture P sequence cycled (one independent stream per GPU)"),
    5: dict(metric="ME+transform+RD megapixels/sec @2160p High10 10-bit EPZS SR=32, CABAC RDO on, 240-MB slices (config 5); "
                   + TIMER,
            disp=(3840, 2160), coded=(3840, 2160), search_mode=3, t8=0, bd=10, slice_mbs=240, rdo=1,
            workload="2160p synthetic YUV420 10-bit (16-bit samples), High 10 (ProfileIDC 110), {sm} "
                     "SearchRange=32, UseHadamard=1, 7 inter block sizes, RDOptimization=1 with SymbolMode=1 (the CABAC "
                     "rate of every candidate on the device), Transform8x8Mode=0, QP 28, IDR + {nf}-picture P sequence "
                     "cycled (one independent stream per GPU)"),
}
# --config 5 --rdo 0: the RDO-off variant of config 5's shape (EPZS + 8x8 transform)
CONFIG5_RDO_OFF = dict(metric="ME+transform megapixels/sec @2160p High10 10-bit EPZS SR=32 + 8x8 transform, 240-MB slices, "
                              "RDO off (config 5 variant); " + TIMER, t8=1, rdo=0,
                       workload="2160p synthetic YUV420 10-bit (16-bit samples), High 10 (ProfileIDC 110), {sm} "
                                "SearchRange=32, Transform8x8Mode=1, UseHadamard=1, 7 inter block sizes, RDO off, QP 28, "
                                "IDR + {nf}-picture P sequence cycled (one independent stream per GPU)")
RDO = 0              # RDOptimization of the run (the config's, or --rdo)
T8_OVERRIDE = None   # --t8: Transform8x8Mode instead of the config's
EPZS_KW = {}         # --epzs-jm10: JM >= 10's EPZS options (docs/JM_SEMANTICS.md items 46, 61, 62)
EPZS_JM10 = dict(epzs_subpel_me=1, epzs_subpel_thres_scale=2, epzs_min_thres_scale=0, epzs_max_thres_scale=2, epzs_dual_refinement=1)
DISP_W, DISP_H = 1920, 1080
W, H = 1920, 1088
SLICE_MBS = 0        # --slice-mbs: SliceMode 1 / SliceArgument (0: one slice per picture)
SR, QP = 32, 28
NMB = (W // 16) * (H // 16)
# algorithmic HBM bytes per coded picture: current 1.5 B/px + reference 1.5 B/px
# (each read once) + reconstruction 1.5 B/px and deblocked reconstruction 1.5 B/px written +
# levels (int16 per sample) 3.0 B/px, plus per-MB side data (MVs, refs, modes, cbp) 80 B/MB; the
# four picture terms double with 16-bit samples (bit depth > 8: 15 B/px)
BD = 8
BYTES_PER_PIXEL = 9.0
SIDE_BYTES_PER_MB = 80
BYTES_PER_FRAME = W * H * BYTES_PER_PIXEL + NMB * SIDE_BYTES_PER_MB
HBM_PEAK_GBS = 8000.0                                    # MI355X_MICROARCH.md (spec)
# integer-search absolute differences per picture (the FFS SAD table)
AD_PER_FRAME = NMB * (2 * SR + 1) ** 2 * 256


def load_module(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def use_config(k, size=None, rdo=None):
    """switch the module-level workload constants to BASELINE.json config k (size: test override;
    rdo: override of the config's RDOptimization, config 5 only)"""
    global DISP_W, DISP_H, W, H, NMB, BYTES_PER_FRAME, AD_PER_FRAME, BD, BYTES_PER_PIXEL, RDO
    c = dict(CONFIGS[k])
    if k == 5 and rdo == 0:
        c.update(CONFIG5_RDO_OFF)
    RDO = c.get("rdo", 0)
    BD = c.get("bd", 8)
    BYTES_PER_PIXEL = 6.0 * (2 if BD > 8 else 1) + 3.0
    (DISP_W, DISP_H), (W, H) = c["disp"], c["coded"]
    if size:
        DISP_W, DISP_H = size
        W, H = (DISP_W + 15) // 16 * 16, (DISP_H + 15) // 16 * 16
    NMB = (W // 16) * (H // 16)
    BYTES_PER_FRAME = W * H * BYTES_PER_PIXEL + NMB * SIDE_BYTES_PER_MB
    AD_PER_FRAME = NMB * (2 * SR + 1) ** 2 * 256
    return c


# v_sad_u8 issue rate measured on MI355X by tools/sad_peak.hip (profiles/r2_sad_peak.json: 62.2
# lane-ops per CU per clock x 256 CUs x 4 absolute differences, scaled to 2.4 GHz); profiles/ does
# not travel to the GPU box, so the figure is kept here
VALU_SAD_MEASURED_TADS = 152.90


def sad_peak():
    """(T AD/s, source) of v_sad_u8 on this chip (measured, tools/sad_peak.hip)."""
    return VALU_SAD_MEASURED_TADS, "measured: v_sad_u8 62.2 lane-ops/CU/clk (tools/sad_peak.hip, profiles/r2_sad_peak.json), at 2.4 GHz"


# VALU issue peak: a wave64 vector instruction issues over 2 cycles on a SIMD-32 (MI355X guide,
# "A wave (64 lanes) ... issues each VALU instruction over 2 cycles"), 4 SIMDs x 256 CUs at 2.4 GHz
VALU_ISSUE_PEAK_TWIS = 256 * 4 * 2.4e9 / 2 / 1e12      # 1.2288 T wave-instructions/s


def exit_status(verified, complete):
    """(exit code, stderr message) of a finished run: 3 when the GPU results differ from the oracle
    (`verified` False), 4 when a rank completed a different number of pictures than --steps in the
    timed region (`complete` False: the timing, not the results, is off), else 0."""
    if verified is False:
        return 3, "bench.py: GPU results differ from the oracle"
    if not complete:
        return 4, "bench.py: a rank completed a different number of pictures than --steps in the timed region"
    return 0, None


# ------------------------------------------------------------------------------------------
# CPU baseline (the oracle: JM restated in C, scalar -O2, one thread per process)
# ------------------------------------------------------------------------------------------
def cpu_one_picture(seed, search_mode, t8=0, dump=None):
    """Seconds the oracle takes for one P picture of the configured size on stream `seed`
    (UnifiedOneForthPix + encode_one_macroblock per MB).  Runs in a child process (bench.py
    --cpu-worker): no GPU is touched.  dump: npz path for the I + P results (the GPU check)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib
    jm = load_module("jmhip", os.path.join(PKG, "jmhip.py"))
    frames = [jm.synth_frame(DISP_W, DISP_H, seed, i, bit_depth=BD) for i in range(2)]
    o = oracle_lib.OracleEncoder(W, H, search_range=SR, search_mode=search_mode, transform_8x8_mode=t8,
                                 slice_mbs=SLICE_MBS, bit_depth=BD, rdo=RDO, **EPZS_KW)
    ires, irec = o.encode(*frames[0], jm.JMH_I_SLICE, QP)
    t0 = time.perf_counter()
    o.set_reference(*irec)
    pres, prec = o.encode(*frames[1], jm.JMH_P_SLICE, QP)
    dt = time.perf_counter() - t0
    o.close()
    if dump:
        np.savez(dump, ires=ires, iy=irec[0], iu=irec[1], iv=irec[2], pres=pres, py=prec[0], pu=prec[1], pv=prec[2])
    return dt


def cpu_workers(n, config, search_mode, size, dump_dir=None):
    """n concurrent child processes (distinct seeds); their per-picture seconds."""
    procs = []
    for k in range(n):
        cmd = [sys.executable, os.path.abspath(__file__), "--cpu-worker", str(k), str(config), str(search_mode),
               f"{size[0]}x{size[1]}"]
        if dump_dir and k == 0:
            cmd.append(os.path.join(dump_dir, "oracle_seed0.npz"))
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True,
                                      env=dict(os.environ, JMH_BENCH_SLICE_MBS=str(SLICE_MBS), JMH_BENCH_RDO=str(RDO),
                                               JMH_BENCH_EPZS10="1" if EPZS_KW else "0", JMH_BENCH_T8=str(T8_OVERRIDE)
                                               if T8_OVERRIDE is not None else "")))
    out = []
    for p in procs:
        s = p.communicate()[0]
        if p.returncode != 0 or not s.split():
            raise RuntimeError(f"cpu worker failed (rc {p.returncode})")
        out.append(float(s.split()[-1]))
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def available_cores():
    """(n, affinity, quota, online): the CPUs this process may use -- its affinity mask, capped by
    the cgroup's CPU quota (cgroup v2 cpu.max or v1 cfs_quota_us / cfs_period_us) where one is set,
    which on a shared box is far below the CPUs it can see -- and the machine's online count."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, aff, quota, os.cpu_count()


def cpu_baseline(config, search_mode, dump_dir, T8):
    """The CPU path timed on this node's host cores: one process on one core (JM is
    single threaded; the reported baseline), and n processes on distinct streams at once
    (aggregate, n = every core available to this process: available_cores).  Worker 0 of the
    one-core run dumps its I + P results for the GPU check."""
    one = cpu_workers(1, config, search_mode, (DISP_W, DISP_H), dump_dir)[0]
    n, aff, quota, online = available_cores()
    many = cpu_workers(n, config, search_mode, (DISP_W, DISP_H))
    mode = {0: "FFS", -1: "full search", 3: "EPZS"}[search_mode] + (" + 8x8 transform" if T8 else "") \
        + (f", {BD}-bit" if BD > 8 else "") + (f", {SLICE_MBS}-MB slices" if SLICE_MBS else "") \
        + (", RDO on (CABAC rate)" if RDO else "")
    return {"value": round(DISP_W * DISP_H / 1e6 / one, 4), "unit": "MP/s", "cores": 1, "kind": "port",
            "sample": f"one {DISP_W}x{DISP_H} P picture (coded {W}x{H}, {NMB} MBs, {mode} SR=32, QP {QP}) incl. "
                      f"quarter-pel interpolation, oracle/liboracle.so -O2 scalar, {one:.1f} s, on {cpu_model()}",
            "all_cores": {"value": round(n * DISP_W * DISP_H / 1e6 / max(many), 4), "unit": "MP/s", "cores": n,
                          "cores_available": {"affinity": aff, "cgroup_quota": quota, "online": online},
                          "sample": f"{n} processes (every core available to this process: affinity {aff}, cgroup "
                                    f"quota {'none' if quota is None else f'{quota:g}'}; {online} online), one P picture "
                                    f"each on distinct streams, concurrently, {max(many):.1f} s wall"}}


def verify_against_oracle(jm, dump, search_mode, t8, device):
    """Encode the CPU baseline's I + P pictures (stream 0) on the GPU and compare every MB result
    and the reconstructions with the oracle's (the dump of the cpu_baseline leg)."""
    import numpy as np
    d = np.load(dump)
    frames = [jm.synth_frame(DISP_W, DISP_H, 0, i, bit_depth=BD) for i in range(2)]
    g = jm.Encoder(W, H, device=device, search_range=SR, search_mode=search_mode, transform_8x8_mode=t8,
                   pipeline_depth=1, slice_mbs=SLICE_MBS, bit_depth=BD, rdo=RDO, **EPZS_KW)
    try:
        ires, irec = g.encode(*frames[0], jm.JMH_I_SLICE, QP)
        g.set_reference(*irec)
        pres, prec = g.encode(*frames[1], jm.JMH_P_SLICE, QP)
    finally:
        g.close()
    ok = ires.tobytes() == d["ires"].tobytes() and pres.tobytes() == d["pres"].tobytes()
    for a, k in zip(irec + prec, ("iy", "iu", "iv", "py", "pu", "pv")):
        ok = ok and np.array_equal(a, d[k])
    return bool(ok)


def read_pmc_traffic(config, search_mode, t8=None, slice_mbs=None):
    """(the pass's record: hbm_bytes_per_mb and, where counted, valu_insts_per_mb of the roofline's
    kernels; source description) from the rocprofv3 PMC passes of tools/pmc_traffic.sh for this
    config, or (None, None).  The latest pass per
    config is kept in tools/pmc_traffic.json (it travels to the GPU box, unlike profiles/); it is
    a committed measurement of an earlier run of the same kernels, not of this run."""
    p = os.path.join(ROOT, "tools", "pmc_traffic.json")
    key = {(2, 0): "2" if os.environ.get("JMH_FLOW", "1") != "0" else "2t", (3, 3): "3", (5, 3): "5",
           (5, 0): "5ffs"}.get((config, search_mode))
    if key is None or (config == 5 and not RDO):
        return None, None
    try:
        with open(p) as f:
            confs = json.load(f)["configs"]
        # a separate pass per Transform8x8Mode where one exists ("5t8": config 5 with 8x8 transform)
        if t8 and key + "t8" in confs:
            key += "t8"
        j = confs[key]
        # only the configuration the pass measured (Transform8x8Mode, slices)
        if ("t8" in j and t8 is not None and j["t8"] != t8) or \
           ("slice_mbs" in j and slice_mbs is not None and j["slice_mbs"] != slice_mbs):
            return None, None
        src = (f"tools/pmc_traffic.json config {key}: {j['kernel']} ({j.get('source', 'rocprofv3 PMC')}; "
               f"{j.get('calibration', 'uncalibrated')})")
        return j, src
    except (OSError, ValueError, KeyError, TypeError):
        return None, None


# ------------------------------------------------------------------------------------------
# the host-buffer path: PCIe-inclusive rate and single-picture latency (reported, not `value`)
# ------------------------------------------------------------------------------------------
def pcie_inclusive(jm, enc, frames, pictures):
    """jmh_frame_push / jmh_frame_pop on host pictures as lencod drives them (source H2D; results
    read in place, the deblocked picture into the caller's planes: D2H), steady state: `depth`
    pictures pushed untimed, then exactly `pictures` pop + push pairs timed (the pipeline stays
    full).  Returns (MP/s, single-picture latency ms on an empty pipeline)."""
    import numpy as np
    enc.sync()
    seq = [tuple(np.ascontiguousarray(p) for p in f) for f in frames[1:]]
    out = (np.empty((enc.h, enc.w), enc.pdt), np.empty((enc.h // 2, enc.w // 2), enc.pdt),
           np.empty((enc.h // 2, enc.w // 2), enc.pdt))
    dbk = (0, 0, 0)
    enc.set_reference_slot(-2)
    enc.push(*seq[0], jm.JMH_P_SLICE, QP, deblock=dbk)   # latency: one picture, empty pipeline
    enc.pop_into(*out)
    latency_ms = enc.timing().total_ms
    for i in range(enc.depth):
        enc.set_reference_slot(-2)
        enc.push(*seq[(1 + i) % len(seq)], jm.JMH_P_SLICE, QP, deblock=dbk)
    t0 = time.perf_counter()
    for i in range(pictures):
        enc.pop_into(*out)
        enc.set_reference_slot(-2)
        enc.push(*seq[(1 + enc.depth + i) % len(seq)], jm.JMH_P_SLICE, QP, deblock=dbk)
    dt = time.perf_counter() - t0
    for _ in range(enc.depth):
        enc.pop_into(*out)
    return pictures * DISP_W * DISP_H / 1e6 / dt, latency_ms, pictures


# ------------------------------------------------------------------------------------------
# launcher: --gpus N without torchrun -> N ranks, one process per GPU
# ------------------------------------------------------------------------------------------
def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def pin_rank(local, nlocal):
    """each stream's host work (launches, result copies) on cores of its own — pin the
    rank to an equal share of the cores this process may use, before anything touches the GPU."""
    cpus = sorted(os.sched_getaffinity(0))
    share = len(cpus) // max(1, nlocal)
    if share < 1:
        return None
    mine = set(cpus[local * share:(local + 1) * share])
    os.sched_setaffinity(0, mine)
    return sorted(mine)


def launch(n):
    """Spawn n ranks of this script (before anything touches the GPU) and return the worst exit
    code.  Rank 0 prints the JSON line."""
    port = str(free_port())
    procs = []
    for k in range(n):
        env = dict(os.environ, RANK=str(k), LOCAL_RANK=str(k), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def main():
    global SLICE_MBS, T8_OVERRIDE
    if len(sys.argv) in (6, 7) and sys.argv[1] == "--cpu-worker":    # child of cpu_baseline()
        SLICE_MBS = int(os.environ.get("JMH_BENCH_SLICE_MBS", "0"))
        w, h = (int(v) for v in sys.argv[5].split("x"))
        c = use_config(int(sys.argv[3]), (w, h), int(os.environ.get("JMH_BENCH_RDO", "0")))
        if os.environ.get("JMH_BENCH_T8", "") != "":
            c["t8"] = int(os.environ["JMH_BENCH_T8"])
        if os.environ.get("JMH_BENCH_EPZS10") == "1":
            EPZS_KW.update(EPZS_JM10)
        print(cpu_one_picture(int(sys.argv[2]), int(sys.argv[4]), c["t8"], sys.argv[6] if len(sys.argv) == 7 else None),
              flush=True)
        return 0
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--frames", type=int, default=60, help="P pictures of the resident source sequence")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive / latency measurement")
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 5),
                    help="BASELINE.json config: 2 = 1080p Baseline FFS (the headline), 3 = 2160p High EPZS + 8x8, "
                         "5 = 2160p High 10 EPZS, CABAC RDO on, 240-MB slices")
    ap.add_argument("--rdo", type=int, default=None, choices=(0, 1),
                    help="config 5: RDOptimization (default 1; 0 = the RDO-off variant with the 8x8 transform)")
    ap.add_argument("--t8", type=int, default=None, choices=(0, 1),
                    help="override the config's Transform8x8Mode (config 5 with RDO on: the 8x8-transform candidates "
                         "and I8MB by RDCost_for_8x8IntraBlocks, docs/JM_SEMANTICS.md item 63)")
    ap.add_argument("--search-mode", type=int, default=None, choices=(0, -1, 3),
                    help="override the config's SearchMode (config 2 variants: -1 full search, 3 EPZS)")
    ap.add_argument("--epzs-jm10", action="store_true",
                    help="EPZS configs: JM >= 10's EPZS options (EPZSSubPelME 1, EPZSSubPelThresScale 2, "
                         "EPZSMin/MaxThresScale 0 / 2, EPZSDualRefinement 1)")
    ap.add_argument("--slice-mbs", type=int, default=None,
                    help="SliceMode 1 with SliceArgument N macroblocks per slice (0: one slice; default: the config's)")
    # test knobs (tests/test_multistream_gpu.py): a smaller picture, a final read-back picture
    ap.add_argument("--size", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--dump", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--no-deblock", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0 and args.gpus > 1:
        return launch(args.gpus)
    world = max(world, 1)
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pinned = pin_rank(local, int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))) if world > 1 else None
    size = tuple(int(v) for v in args.size.split("x")) if args.size else None
    if args.rdo is not None and args.config != 5:
        ap.error("--rdo applies to --config 5")
    cfg = use_config(args.config, size, args.rdo)
    if args.t8 is not None:
        if args.t8 and args.config == 2:
            ap.error("--t8 1 needs a High profile config (3 or 5)")
        T8_OVERRIDE = args.t8
        if cfg["t8"] != args.t8:
            cfg["workload"] = cfg["workload"].replace(f"Transform8x8Mode={cfg['t8']}", f"Transform8x8Mode={args.t8}")
            cfg["metric"] = cfg["metric"] + (" + 8x8 transform" if args.t8 else " (4x4 transform)")
        cfg["t8"] = args.t8
    SLICE_MBS = max(0, cfg.get("slice_mbs", 0) if args.slice_mbs is None else args.slice_mbs)
    search_mode = cfg["search_mode"] if args.search_mode is None else args.search_mode
    if search_mode != cfg["search_mode"]:   # the metric names the search the line measured
        own = cfg.get("metric_sm", {0: "FFS", -1: "FullSearch", 3: "EPZS"}[cfg["search_mode"]])
        cfg["metric"] = cfg["metric"].replace(own, {0: "FFS", -1: "FullSearch SearchMode=-1", 3: "EPZS"}[search_mode], 1)
    if args.epzs_jm10:
        if search_mode != 3:
            ap.error("--epzs-jm10 applies to EPZS (SearchMode 3)")
        EPZS_KW.update(EPZS_JM10)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    jm = load_module("jmhip", os.path.join(PKG, "jmhip.py"))
    streams = load_module("jmh_streams", os.path.join(PKG, "streams.py"))
    ndev = jm.load().jmh_device_count()
    if ndev <= 0:
        raise SystemExit("bench.py: no HIP device")
    device = local % ndev
    frames = [jm.synth_frame(DISP_W, DISP_H, rank, i, bit_depth=BD) for i in range(args.frames + 1)]
    enc = jm.Encoder(W, H, device=device, search_range=SR, search_mode=search_mode, slots=len(frames),
                     kernel_timing=True, transform_8x8_mode=cfg["t8"], slice_mbs=SLICE_MBS, bit_depth=BD, rdo=RDO, **EPZS_KW)
    stream = streams.PStream(enc, frames, QP, deblock=None if args.no_deblock else (0, 0, 0))
    dt = streams.timed_run(stream, args.steps, args.warmup, dist, on_start=enc.timing)   # on_start resets the event sums
    tm = enc.timing()                                     # event sums of the timed steps only

    host = None
    if not args.no_host_path and size is None and not args.no_deblock:
        host = pcie_inclusive(jm, enc, frames, max(120, 3 * enc.depth))
    if args.dump:                                         # test: one read-back picture after the chain
        import numpy as np
        enc.set_reference_slot(stream.ref_slot)
        res, rec = enc.encode(*frames[1], jm.JMH_P_SLICE, QP, deblock=stream.deblock)
        np.savez(os.path.join(args.dump, f"rank{rank}.npz"), res=res, y=rec[0], u=rec[1], v=rec[2],
                 slots=np.array(stream.slots_used), device=device, warmup=stream.warmup_steps)
    mine = {"rank": rank, "device": device, "dt": dt, "pictures_completed": tm.pictures_done,
            "cpus": None if pinned is None else f"{pinned[0]}-{pinned[-1]}" if pinned == list(range(pinned[0], pinned[-1] + 1))
            else ",".join(map(str, pinned))}
    everyone = [mine]
    if dist is not None:
        everyone = [None] * world
        dist.all_gather_object(everyone, mine)
    complete = all(e["pictures_completed"] == args.steps for e in everyone)
    if rank != 0:
        if dist is not None:
            dist.barrier()
        enc.sync()                                        # complete the pictures still in flight
        enc.close()
        return 0 if complete else 4

    value = world * args.steps * DISP_W * DISP_H / 1e6 / dt
    pictures = max(1, tm.pictures)
    FLOW = tm.flow_launches > 0                          # dataflow: one k_mb_flow launch per segment of ticks
    an_per_pic = (tm.flow_launches if FLOW else tm.ticks) / pictures   # tick model: one k_mb_analyse + one k_mb_final per tick
    mb_ms_pic = tm.mb_ms / pictures
    # the sampled launches' HIP events (every 32nd tick) add a few us per launch; the wavefront
    # brackets (one event pair per run of ticks) do not.  The per-launch figures are scaled so that
    # the sampled launches of a tick sum to the bracketed wavefront time per tick (never above it):
    # k_mb_analyse 93.8 us raw vs 90.0 us in rocprof's kernel trace (profiles/r6h_*)
    an_raw_ms = tm.analyse_ms / max(1, tm.analyse_launches)
    fin_raw_ms = 0.0 if RDO or FLOW else tm.final_ms / max(1, tm.final_launches)
    ev_scale = min(1.0, mb_ms_pic / an_per_pic / (an_raw_ms + fin_raw_ms)) if an_raw_ms + fin_raw_ms > 0 else 1.0
    an_launch_ms, fin_launch_ms = an_raw_ms * ev_scale, fin_raw_ms * ev_scale
    # MBs of all pictures in flight per tick, or per dataflow segment
    mbs_per_launch = tm.flow_mbs / tm.flow_launches if FLOW else tm.tick_mbs / max(1, tm.ticks)
    bytes_per_launch = BYTES_PER_FRAME / NMB * mbs_per_launch
    achieved_gbs = bytes_per_launch / (an_launch_ms * 1e-3) / 1e9
    ad_per_launch = AD_PER_FRAME / NMB * mbs_per_launch
    achieved_tads = ad_per_launch / (an_launch_ms * 1e-3) / 1e12
    peak_tads, peak_src = sad_peak()
    pmc_rec, pmc_src = read_pmc_traffic(args.config, search_mode, cfg["t8"], SLICE_MBS)
    pmc = pmc_rec["hbm_bytes_per_mb"] if pmc_rec else None
    valu_mb = pmc_rec.get("valu_insts_per_mb") if pmc_rec else None
    sm_name = {0: "FFS SearchMode=0", -1: "full search SearchMode=-1", 3: "EPZS SearchMode=3"}[search_mode]
    ffs = search_mode == 0
    an_name = ("k_mb_flow" if FLOW else "k_rdo_inter+k_rdo_intra+k_rdo_final" if RDO else
               ("k_mb_analyse+k_mb_intra8" if cfg["t8"] else "k_mb_analyse") if ffs else
               ("k_mb_epzs" if search_mode == 3 else "k_mb_me_full") + "+k_mb_intra")
    hbm = {
        "bound": "hbm",
        "achieved": round(achieved_gbs, 3),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved_gbs / HBM_PEAK_GBS, 6),
        "traffic": round(pmc * mbs_per_launch) if pmc else None,
        "traffic_source": pmc_src,
        "algorithmic_bytes_per_launch": round(bytes_per_launch),
    }
    launch_info = {
        "kernel": an_name.replace("+", " + ") + (" (the dataflow wavefront: one launch per segment of ticks, one workgroup "
                                                  "per macroblock running its search, intra decisions and final)" if FLOW else
                                                  " (the tick's RD launches: inter and intra on two streams, then final; "
                                                  "the span of the three)" if RDO else
                                                  "" if ffs and not cfg["t8"] else " (the tick's analysis launches)"),
        "avg_launch_ms": round(an_launch_ms, 5),
        "avg_launch_ms_events_raw": round(an_raw_ms, 5),
        "event_scale": round(ev_scale, 4),
        "launches_per_picture": round(an_per_pic, 2),
        "mbs_per_launch": round(mbs_per_launch, 1),
    }
    # the issue view: the kernels' VALU wave-instructions per MB (the committed PMC pass) x the MBs
    # of a launch / the launch time, against the chip's VALU issue rate
    issue = None
    if valu_mb:
        achieved_twis = valu_mb * mbs_per_launch / (an_launch_ms * 1e-3) / 1e12
        issue = dict(bound="valu-issue", achieved=round(achieved_twis, 4), peak=round(VALU_ISSUE_PEAK_TWIS, 4),
                     unit="T VALU wave-instructions/s", frac=round(achieved_twis / VALU_ISSUE_PEAK_TWIS, 4),
                     valu_insts_per_mb=valu_mb, valu_insts_per_mb_kernels=pmc_rec.get("valu_kernels"),
                     sad_floor_insts_per_mb=round((2 * SR + 1) ** 2 * 256 / 4 / 64) if ffs else None,
                     traffic=hbm["traffic"], traffic_source=pmc_src,
                     traffic_over_algorithmic=round(hbm["traffic"] / bytes_per_launch, 2) if hbm["traffic"] else None,
                     peak_source="MI355X guide: a wave64 VALU instruction issues over 2 cycles on a SIMD-32; "
                                 "256 CUs x 4 SIMDs x 2.4 GHz / 2",
                     note="VALU wave-instructions per MB from the committed PMC pass (SQ_INSTS_VALU, " + str(pmc_src)
                          + ") x the MBs of a launch / this run's launch time")
    if ffs:   # config 2: the FFS SAD table binds -> VALU roofline; HBM beside it
        roofline = dict(bound="valu", achieved=round(achieved_tads, 4), peak=round(peak_tads, 2),
                        unit="T abs-diff/s", frac=round(achieved_tads / peak_tads, 5),
                        traffic=hbm["traffic"], traffic_source=pmc_src, peak_source=peak_src,
                        algorithmic_ad_per_launch=round(ad_per_launch), **launch_info, hbm=hbm, issue=issue)
    elif issue:   # EPZS / RD searches: bound by instruction issue along dependent chains, not HBM
        roofline = dict(issue, **launch_info, hbm=hbm)
    else:
        roofline = dict(hbm, **launch_info)
    out = {
        "metric": cfg["metric"],
        "timer": TIMER + "; SURVEY §8d's submit-to-host-visible timer: host_path.pcie_inclusive_mp_s",
        "value": round(value, 3),
        "unit": "MP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16" if BD > 8 else "u8",
        "data": "synthetic",
        "config": {
            "workload": cfg["workload"].replace("{sm}", sm_name).replace("{nf}", str(args.frames))
                        + (f", SliceMode=1 SliceArgument={SLICE_MBS} ({-(-NMB // SLICE_MBS)} slices per picture)"
                           if SLICE_MBS else "")
                        + (", JM >= 10 EPZS options: EPZSSubPelME=1 EPZSSubPelThresScale=2 EPZSMinThresScale=0 "
                           "EPZSMaxThresScale=2 EPZSDualRefinement=1" if EPZS_KW else ""),
            "global_batch": world,
            "parallelism": f"streams{world}",
            "pipeline_depth": enc.depth,
            "devices": [e["device"] for e in everyone],
        },
        "timed_region": {
            "warmup_steps_run": stream.warmup_steps,
            "pictures_completed": [e["pictures_completed"] for e in everyone],
            "per_rank_s": [round(e["dt"], 5) for e in everyone],
            "per_rank_mp_s": [round(args.steps * DISP_W * DISP_H / 1e6 / e["dt"], 3) for e in everyone],
            "per_rank_cpus": [e["cpus"] for e in everyone],
            "note": "steady state: the pipeline is full at both ends (barrier + wait for the issued launches, "
                    "pictures in flight are not drained); exactly `steps` pictures complete inside",
        },
        "roofline": roofline,
        # per-launch averages (sampled every 32nd tick, scaled to the bracketed wavefront time: see
        # ev_scale) x launches per picture; RDO on: the span of a tick's three RD launches
        "kernel_ms_per_picture": {"wavefront": round(mb_ms_pic, 4),
                                  an_name + (" (tick span)" if RDO else ""): round(an_launch_ms * an_per_pic, 4),
                                  "k_mb_final": None if RDO else round(fin_launch_ms * an_per_pic, 4),
                                  "note": "HIP events on the kernels' stream; the sampled per-launch averages are "
                                          "scaled by event_scale so that a tick's launches sum to the bracketed "
                                          "wavefront time per tick (the sampling events add a few us per launch)"},
        "host_path": None if host is None else {
            "pcie_inclusive_mp_s": round(host[0], 3),
            "single_picture_latency_ms": round(host[1], 3),
            "note": "jmh_frame_push/pop with host pictures as lencod drives them: source H2D (packed into "
                    "pinned staging), results/recon/deblocked D2H on the copy stream, the results read in "
                    "place and the deblocked picture copied into the caller's planes; steady state, "
                    "exactly `pictures` pop+push pairs timed; latency = one picture on an empty pipeline "
                    "(fill + drain)",
            "pictures": host[2],
        },
        "complete": complete,                             # exactly --steps pictures inside the timed region
        "verified": None,                                 # the oracle comparison (cpu_baseline leg)
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        with tempfile.TemporaryDirectory() as tmp:
            out["cpu_baseline"] = cpu_baseline(args.config, search_mode, tmp, cfg["t8"])
            out["verified"] = verify_against_oracle(jm, os.path.join(tmp, "oracle_seed0.npz"), search_mode, cfg["t8"],
                                                    device)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
    enc.sync()                                            # complete the pictures still in flight
    enc.close()
    rc, msg = exit_status(out["verified"], complete)
    if msg:
        print(msg, file=sys.stderr)
    return rc


if __name__ == "__main__":
    sys.exit(main())
