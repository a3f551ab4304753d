#!/usr/bin/env python3
"""Summarise one k_mb_flow launch's per-ticket stamps (JMH_FLOW_PROF=<launch>, JMH_FLOW_PROF_OUT=file).

Per workgroup (ticket order): start -> dependencies met (+acquire) -> analysis done -> final done ->
flag stored.  Prints the phase durations, how many workgroups were resident / waiting / working
over time, and the share of slot time spent waiting."""
import sys

import numpy as np


def load(path):
    raw = open(path, "rb").read()
    n, khz, mbw, mbh = np.frombuffer(raw[:32], np.uint64).astype(np.int64)
    st = np.frombuffer(raw[32:32 + 48 * n], np.uint64).reshape(n, 6)
    items = np.frombuffer(raw[32 + 48 * n:32 + 48 * n + 4 * n], np.uint32)
    return st, items, 1e3 / khz, mbw, mbh


def main(path):
    st, items, us, mbw, mbh = load(path)
    n = len(st)
    t = (st[:, :5].astype(np.int64) - int(st[:, 0].min())) * us
    hw = (st[:, 5] >> 32).astype(np.int64)
    wait, ana, fin, rel = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 4] - t[:, 3]
    span = t[:, 4].max()
    pct = lambda a: f"mean {a.mean():6.1f}  p50 {np.percentile(a, 50):6.1f}  p90 {np.percentile(a, 90):6.1f}  max {a.max():6.1f}"
    print(f"launch: {n} MBs, span {span:.1f} us -> {n / span:.2f} MBs/us ({n / span * 1e6 / 8160 * 2.0736:.1f} MP/s at 1080p)")
    print(f"wait (claim -> deps met + acquire): {pct(wait)}")
    print(f"analysis (search + intra):         {pct(ana)}")
    print(f"final (+ I16/chroma decisions):    {pct(fin)}")
    print(f"release + flag:                    {pct(rel)}")
    busy = (t[:, 4] - t[:, 0]).sum()
    print(f"slot time: waiting {wait.sum() / busy * 100:.1f} %, analysis {ana.sum() / busy * 100:.1f} %, "
          f"final {fin.sum() / busy * 100:.1f} %, release {rel.sum() / busy * 100:.1f} %")
    # residency over time
    grid = np.linspace(0, span, 200)
    res = np.array([((t[:, 0] <= g) & (t[:, 4] > g)).sum() for g in grid])
    wt = np.array([((t[:, 0] <= g) & (t[:, 1] > g)).sum() for g in grid])
    mid = (grid > span * 0.1) & (grid < span * 0.9)
    print(f"resident workgroups (middle 80 %): mean {res[mid].mean():.0f} (max {res.max()}), of them waiting {wt[mid].mean():.0f}")
    # gaps: a workgroup's start vs the previous workgroup's end on the same slot is not recorded; approximate
    # the dispatch refill by the start-time spread of consecutive tickets
    d = np.diff(t[:, 0])
    print(f"ticket start spacing: mean {d.mean() * 1000:.0f} ns, p99 {np.percentile(d, 99) * 1000:.0f} ns")
    # per MB index of the tick: the waits of MBs by their dependency kind
    e = items >> 24
    print("entries in the launch:", sorted(set(e.tolist())))
    xcc = (hw >> 16) & 15
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  XCC {x}: {m.sum()} MBs, wait {wait[m].mean():.1f}, analysis {ana[m].mean():.1f}, final {fin[m].mean():.1f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "flow_prof.bin")
