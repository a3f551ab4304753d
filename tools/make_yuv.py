#!/usr/bin/env python3
"""Write a planar I420 file of the deterministic synthetic sequence (the lencod 'synthetic:<seed>'
source, host/yuv.c jm_synth_frame), so lencod end-to-end runs read a file like JM does instead of
timing the generator:   python tools/make_yuv.py OUT W H FRAMES [SEED]"""
import importlib.util
import os
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("jmhip", os.path.join(ROOT, "h264-jm-commentary_amd", "jmhip.py"))
jm = importlib.util.module_from_spec(spec)
spec.loader.exec_module(jm)


def frame(args):
    w, h, seed, i = args
    y, u, v = jm.synth_frame(w, h, seed, i)
    return y[:h, :w].tobytes() + u[:h // 2, :w // 2].tobytes() + v[:h // 2, :w // 2].tobytes()


if __name__ == "__main__":
    out, w, h, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    seed = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    with Pool(min(8, os.cpu_count() or 1)) as pool, open(out, "wb") as f:
        for buf in pool.imap(frame, [(w, h, seed, i) for i in range(n)]):
            f.write(buf)
