#!/usr/bin/env python3
"""Bound a dataflow schedule for config 2 by list-scheduling simulation.

Model (calibrated on the measured steady-state tick, DESIGN.md §5.1, JMH_BLOCK_PROF):
- 256 CUs x 2 slots (k_mb_analyse: 78 KB LDS and 123 VGPRs per 512-thread workgroup);
- one MB's search alone on a CU takes W_S us (55.7: JMH_PHASE_PROF single MB); two workgroups on
  one CU share it: the older runs at rate R_OLD, the younger at R_YOUNG (fitted so that a pair
  started together ends at p50 57.8 / max 79 us, the measured steady tick);
- the rest of a macroblock (Intra16x16 / chroma decision + k_mb_final's work) is W_F us of work
  at the same rates; every MB's search work is drawn per MB from a spread that reproduces the
  tick's p50..max range;
- dataflow: a free slot claims the next MB in tick order (the order the host issues ticks, lag
  PIPE_LAG = 16), waits (holding its slot) until its left and top-right neighbours (top at the
  right edge) and the reference picture's MB (x+5, y+5) (clamped) are done, then runs search +
  rest on that slot; SYNC us of flag hand-off per MB;
- tick model (for calibration): every tick runs its MBs two per CU, the tick ends with the
  slowest, then a final launch (FIN us) and the launch gaps (GAP us).

Prints the steady-state picture period and MP/s of both models.
"""
import argparse
import heapq
import random

MBW, MBH = 120, 68
LAG = 16


def diag_list():
    nd = MBW - 1 + 2 * (MBH - 1) + 1
    diags = [[] for _ in range(nd)]
    for y in range(MBH):
        for x in range(MBW):
            diags[x + 2 * y].append((x, y))
    return diags


def tick_order(npics):
    """MB (pic, x, y) lists per tick, as jmhip_abi.hip issue_tick does (lag 16, unbounded PMAX)."""
    diags = diag_list()
    nd = len(diags)
    stage = [0] * npics
    ticks = []
    while True:
        act = []
        for p in range(npics):
            if stage[p] >= nd:
                continue
            if p > 0 and stage[p - 1] < nd and stage[p - 1] - stage[p] < LAG:
                continue
            act.append(p)
        if not act:
            break
        t = []
        for p in act:
            t += [(p, x, y) for (x, y) in diags[stage[p]]]
            stage[p] += 1
        ticks.append(t)
    return ticks


def sample_work(rng, a):
    # search work spread: most MBs near the mean, a tail ~8 % longer (the tick's p90/max)
    return a.ws * (1.0 + a.spread * (rng.random() ** 3))


def sim_dataflow(a, ticks, npics):
    rng = random.Random(1)
    order = [m for t in ticks for m in t]
    done = {}
    work = {m: sample_work(rng, a) + a.wf for m in order}
    # per CU: list of [mb, remaining, start_time, running(bool)]
    ncu = 256
    cus = [[] for _ in range(ncu)]
    now = 0.0
    nxt = 0
    ev = []
    ver = [0] * ncu

    def deps(m):
        p, x, y = m
        d = []
        if x > 0:
            d.append((p, x - 1, y))
        if y > 0:
            d.append((p, x + 1, y - 1) if x + 1 < MBW else (p, x, y - 1))
        if p > 0:
            d.append((p - 1, min(x + 5, MBW - 1), min(y + 5, MBH - 1)))
        return d

    waiters = {}

    def rates(c):
        run = [w for w in cus[c] if w[3]]
        if len(run) == 1:
            return {id(run[0]): 1.0}
        if len(run) == 2:
            o, y = sorted(run, key=lambda w: w[2])
            return {id(o): a.r_old, id(y): a.r_young}
        return {}

    last = [0.0] * ncu

    def advance(c, t):
        r = rates(c)
        dt = t - last[c]
        for w in cus[c]:
            if w[3]:
                w[1] -= r[id(w)] * dt
        last[c] = t

    def schedule(c):
        ver[c] += 1
        r = rates(c)
        best = None
        for w in cus[c]:
            if w[3]:
                tt = last[c] + max(w[1], 0) / r[id(w)]
                if best is None or tt < best:
                    best = tt
        if best is not None:
            heapq.heappush(ev, (best, c, ver[c]))

    def try_start(c, w):
        m = w[0]
        if all(d in done for d in deps(m)):
            w[3] = True
            w[2] = now
            w[1] += a.sync
            return True
        for d in deps(m):
            if d not in done:
                waiters.setdefault(d, []).append((c, w))
                break
        return False

    def claim(c):
        nonlocal nxt
        if nxt >= len(order):
            return
        m = order[nxt]
        nxt += 1
        w = [m, work[m], now, False]
        cus[c].append(w)
        try_start(c, w)

    for c in range(ncu):
        claim(c)
        claim(c)
        schedule(c)
    pic_done = {}
    cnt = {}
    per_pic = MBW * MBH
    while ev:
        t, c, v = heapq.heappop(ev)
        if v != ver[c]:
            continue
        now = t
        advance(c, now)
        fin = [w for w in cus[c] if w[3] and w[1] <= 1e-9]
        for w in fin:
            cus[c].remove(w)
            m = w[0]
            done[m] = now
            cnt[m[0]] = cnt.get(m[0], 0) + 1
            if cnt[m[0]] == per_pic:
                pic_done[m[0]] = now
            for (c2, w2) in waiters.pop(m, []):
                if w2 in cus[c2] and not w2[3]:
                    advance(c2, now)
                    if try_start(c2, w2):
                        schedule(c2)
            claim(c)
        schedule(c)
    ts = [pic_done[p] for p in sorted(pic_done)]
    k0, k1 = npics // 3, npics - 3
    return (ts[k1] - ts[k0]) / (k1 - k0)


def sim_ticks(a, ticks, npics):
    rng = random.Random(1)
    t = 0.0
    pic_end = {}
    for tk in ticks:
        n = len(tk)
        ws = [sample_work(rng, a) for _ in tk]
        # two per CU: pairs; the older at r_old until it ends, the younger at r_young then alone
        span = 0.0
        for i in range(0, n, 2):
            if i + 1 < n:
                w1, w2 = ws[i], ws[i + 1]
                t1 = w1 / a.r_old
                rem = w2 - a.r_young * t1
                t2 = t1 + max(rem, 0) if rem > 0 else w2 / a.r_young
                span = max(span, t1, t2)
            else:
                span = max(span, ws[i])
        t += span + a.fin + a.gap
        for (p, x, y) in tk:
            pic_end[p] = t
    ts = [pic_end[p] for p in sorted(pic_end)]
    k0, k1 = npics // 3, npics - 3
    return (ts[k1] - ts[k0]) / (k1 - k0), len(ticks)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", type=float, default=55.7)
    ap.add_argument("--spread", type=float, default=0.12)
    ap.add_argument("--wf", type=float, default=11.0, help="I16/chroma + final work per MB, us alone")
    ap.add_argument("--r-old", type=float, default=0.96)
    ap.add_argument("--r-young", type=float, default=0.60)
    ap.add_argument("--sync", type=float, default=4.0, help="flag hand-off per MB, us")
    ap.add_argument("--fin", type=float, default=17.0)
    ap.add_argument("--gap", type=float, default=5.0)
    ap.add_argument("--pics", type=int, default=24)
    a = ap.parse_args()
    ticks = tick_order(a.pics)
    pt, nt = sim_ticks(a, ticks, a.pics)
    mp = 1920 * 1080 / 1e6
    print(f"tick model:     {pt:8.1f} us / picture  ({pt / 16:.1f} us / tick)  {mp / pt * 1e6:8.1f} MP/s")
    pd = sim_dataflow(a, ticks, a.pics)
    print(f"dataflow model: {pd:8.1f} us / picture  {mp / pd * 1e6:8.1f} MP/s  ({(pt / pd - 1) * 100:+.1f} %)")


if __name__ == "__main__":
    main()
