// jmh_intra8.h — the Intra8x8 macroblock decision of one MB on 256 threads (k_mb_intra8 in
// jmh_intra8.hip; k_mb_intra in jmh_analyse.hip for ticks whose motion search has its own kernel).
#pragma once
#include "jmh_common.h"

template <class pel>
struct I8S {
    pel org[256];
    alignas(4) pel rec[256];             // this MB's Intra8x8 reconstruction, block by block
    int raw[25], av[25], f[25];          // reference edge: [7 - y] left, [8] corner, [9 + x] top
    int mcost[9];
    int modes[4];
    int nz[4];
};

// mi: the MB's index in the tick; every thread of the 256-thread workgroup calls this.  pel:
// uint8_t or uint16_t samples (High 10: QP'Y = QPY + QpBdOffsetY, Clip1Y, DC 1 << (BitDepthY - 1))
template <class pel>
__device__ __forceinline__ void intra8_mb(const TickArgs &t, I8S<pel> &s, int mi) {
    const int tid = threadIdx.x;
    const int e = tick_entry(t, mi);
    const DevParams d = tick_params(t, e);
    const int mby = d.y_min + (mi - t.pre[e]), mbx = d.diag - 2 * mby;
    const int pix_x = 16 * mbx, pix_y = 16 * mby, W = d.W, W4 = d.W >> 2;
    const MbAvail mav = intra_avail(d, mbx, mby);
    const bool avL = mav.L, avT = mav.T, avTL = mav.TL, avTR = mav.TR;
    const int lambda = d.lambda_mode, qp = d.qp + d.qpbd, had = d.use_hadamard;
    const pel *orgY = spl<pel>(d.orgY), *recY = spl<pel>(d.recY);
    const int q_bits = 16 + qp / 6;
    const int qp_const = q_round(d.qsel, q_bits);   // items 1, 45
    const int wv = tid >> 6, l = tid & 63, x = l & 7, y = l >> 3;
    MbScratch *sc = d.scr + mby * d.mbw + mbx;

    s.org[tid] = orgY[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)];
    int total = 6 * lambda, cbp = 0;                 // (int)floor(6*lambda + 0.4999), once per MB
    for (int b8 = 0; b8 < 4; b8++) {
        const int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
        const bool left = bx ? true : avL, up = by ? true : avT;
        const bool ul = bx && by ? true : bx ? avT : by ? avL : avTL;
        const bool ur = b8 == 0 ? avT : b8 == 1 ? avTR : b8 == 2;
        __syncthreads();                             // s.org, the previous block's s.rec / s.modes
        if (tid < 25) {
            int xm, ym;
            bool a;
            if (tid < 8) { xm = bx - 1; ym = by + 7 - tid; a = left; }
            else if (tid == 8) { xm = bx - 1; ym = by - 1; a = ul; }
            else { const int xx = tid - 9; xm = bx + (xx < 8 || ur ? xx : 7); ym = by - 1; a = up; }
            int v = 0;
            if (a) v = (xm >= 0 && xm < 16 && ym >= 0) ? s.rec[ym * 16 + xm] : recY[(pix_y + ym) * W + pix_x + xm];
            s.raw[tid] = v; s.av[tid] = a;
        }
        __syncthreads();
        if (tid < 25 && s.av[tid]) {                 // 8.3.2.2.1: [1 2 1] along the edge
            const int c = s.raw[tid];
            const int lo = tid > 0 && s.av[tid - 1] ? s.raw[tid - 1] : c, hi = tid < 24 && s.av[tid + 1] ? s.raw[tid + 1] : c;
            s.f[tid] = (lo + 2 * c + hi + 2) >> 2;
        }
        // predIntra8x8PredMode (8.3.2.1): this MB's earlier blocks, else the neighbour's 4x4 mode
        int ma = -1, mb = -1;
        if (bx) ma = s.modes[b8 - 1];
        else if (avL) ma = d.ipred[(4 * mby + (by >> 2)) * W4 + 4 * mbx - 1];
        if (by) mb = s.modes[b8 - 2];
        else if (avT) mb = d.ipred[(4 * mby - 1) * W4 + 4 * mbx + (bx >> 2)];
        const int mpm = (ma < 0 || mb < 0) ? 2 : min(ma, mb);
        __syncthreads();
        int st = 0, sl = 0;
        for (int i = 0; i < 8; i++) { st += up ? s.f[9 + i] : 0; sl += left ? s.f[i] : 0; }
        const int dcv = up && left ? (st + sl + 8) >> 4 : up ? (st + 4) >> 3 : left ? (sl + 4) >> 3 : (d.maxv + 1) >> 1;
        const int ov = s.org[(by + y) * 16 + bx + x];
        for (int m = wv; m < 9; m += 4) {
            const bool ok = m == 2 || ((m == 0 || m == 3 || m == 7) && up) || ((m == 1 || m == 8) && left) ||
                            ((m == 4 || m == 5 || m == 6) && up && left && ul);
            int cost = BIGCOST;
            if (ok) cost = wave_satd8(ov - i8_pred_px(s.f, dcv, m, x, y), l, had) + (m == mpm ? 0 : 4 * lambda);
            if (l == 0) s.mcost[m] = cost;
        }
        __syncthreads();
        int best = 0, bcost = s.mcost[0];
        for (int m = 1; m < 9; m++)
            if (s.mcost[m] < bcost) { bcost = s.mcost[m]; best = m; }
        total += bcost;
        if (wv == 0) {                               // dct_luma8x8 of the winner + reconstruction
            const int p = i8_pred_px(s.f, dcv, best, x, y);
            const int c = wave_fwd8x8(ov - p, l);
            int lev, dq, cost;
            const unsigned long long nz = wave_quant8(c, l, qp, qp_const, lev, dq, cost);
            s.rec[(by + y) * 16 + bx + x] = (pel)wave_inv8x8(dq, l, p, d.maxv);
            sc->i8lev[il_blk(b8, l)][l >> 2] = (int16_t)lev;
            if (l == 0) { s.modes[b8] = best; s.nz[b8] = nz != 0; }
        }
    }
    __syncthreads();
    spl<pel>(sc->i8rec)[tid] = s.rec[tid];
    if (tid == 0) {
        for (int b = 0; b < 4; b++) cbp |= s.nz[b] << b;
        sc->i8cost = total;
        sc->i8cbp = cbp;
        sc->i8modes = s.modes[0] | s.modes[1] << 4 | s.modes[2] << 8 | s.modes[3] << 12;
    }
}


