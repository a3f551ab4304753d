#!/usr/bin/env python3
"""Debug: config 3 (2160p EPZS + 8x8) ms per picture against the pipeline depth (pictures in flight).
    python tools/depth_sweep.py [depth ...]"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "h264-jm-commentary_amd")


def load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


jm = load("jmhip", os.path.join(PKG, "jmhip.py"))
streams = load("jmh_streams", os.path.join(PKG, "streams.py"))
W, H = int(os.environ.get("W", "3840")), int(os.environ.get("H", "2160"))
sm, t8 = int(os.environ.get("SEARCH_MODE", "3")), int(os.environ.get("T8", "1"))
frames = [jm.synth_frame(W, H, 0, i) for i in range(3)]
for depth in [int(a) for a in sys.argv[1:]] or [20, 24, 27, 30, 33]:
    enc = jm.Encoder(W, H, search_range=32, search_mode=sm, slots=3, kernel_timing=True, transform_8x8_mode=t8,
                     pipeline_depth=depth)
    st = streams.PStream(enc, frames, 28)
    dt = streams.timed_run(st, 150, 40, None, on_start=enc.timing)
    tm = enc.timing()
    print(f"depth {depth}: {dt / 150 * 1e3:.2f} ms/picture, {tm.tick_mbs / max(1, tm.ticks):.0f} MBs/tick, "
          f"{tm.ticks / max(1, tm.pictures):.2f} ticks/picture, analyse {tm.analyse_ms / max(1, tm.analyse_launches):.3f} ms/tick",
          flush=True)
    enc.close()
