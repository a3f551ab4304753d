// jmh_i4.h — Mode_Decision_for_Intra4x4Macroblock [J] on one wave per 4x4 block: the state of an
// MB's Intra4x4 decision (IntraS) and i4_block, shared by k_mb_analyse (the wavefront's intra roles
// and the P macroblocks' intra slots) and tools/i4_bench.hip (its latency on one wave).
#pragma once
#include "jmh_common.h"
#include "jmh_intra.h"

template <class pel>
struct IntraS {
    alignas(4) pel org[256];
    alignas(4) pel rec[256];
    Border bd;
    IntraNb<pel> nb;
    int8_t ipred_cur[16];
    int part[2][4];                           // per I4 wave: cost, cbp, blk mask
};

// ======================================================================================
//  role 0: Intra4x4 (Mode_Decision_for_Intra4x4Macroblock) in 10 diagonal steps
// ======================================================================================
template <class pel>
__device__ __forceinline__ int lpix(const IntraS<pel> &s, int x, int y) {
    if (y < 0) return s.nb.rtop[x + 1];
    if (x < 0) return s.nb.rleft[y];
    return s.rec[16 * y + x];
}

// lane_fwd4x4 / lane_inv4x4 with the row gathers as quad DPP broadcasts (the four samples of
// row y of a 16-lane group are one quad); the column gathers stay ds_bpermute (whole quads active);
// the outputs of each butterfly stage by fwd_tap / inv_tap (jmh_common.h)
__device__ __forceinline__ int quad_fwd4x4(int r, int l) {
    const int y = l >> 2, x = l & 3;
    const int v0 = dpp<0x00>(r), v1 = dpp<0x55>(r), v2 = dpp<0xAA>(r), v3 = dpp<0xFF>(r);
    const int t = fwd_tap(v0 + v3, v1 + v2, v1 - v2, v0 - v3, x);
    const int u0 = g16(t, x), u1 = g16(t, 4 + x), u2 = g16(t, 8 + x), u3 = g16(t, 12 + x);
    return fwd_tap(u0 + u3, u1 + u2, u1 - u2, u0 - u3, y);
}
__device__ __forceinline__ int quad_inv4x4(int dq, int l, int pred, int maxv) {
    const int y = l >> 2, x = l & 3;
    const int d0 = dpp<0x00>(dq), d1 = dpp<0x55>(dq), d2 = dpp<0xAA>(dq), d3 = dpp<0xFF>(dq);
    const int t = inv_tap(d0 + d2, d0 - d2, (d1 >> 1) - d3, d1 + (d3 >> 1), x);
    const int f0 = g16(t, x), f1 = g16(t, 4 + x), f2 = g16(t, 8 + x), f3 = g16(t, 12 + x);
    const int o = inv_tap(f0 + f2, f0 - f2, (f1 >> 1) - f3, f1 + (f3 >> 1), y);
    return iclip(0, maxv, (o + (pred << 6) + 32) >> 6);
}

// the Intra4x4 prediction table entries of lane 4m + y (mode m < 9, block row y): c_i4tab of its
// four samples, two 16-bit entries per dword (i4_block)
__device__ __forceinline__ void i4_tabrow(int lane, int (&tabr)[2]) {
    const int m = lane >> 2, y = lane & 3;
    tabr[0] = m < 9 ? (int)(c_i4tab[m][4 * y] | (uint32_t)c_i4tab[m][4 * y + 1] << 16) : 0;
    tabr[1] = m < 9 ? (int)(c_i4tab[m][4 * y + 2] | (uint32_t)c_i4tab[m][4 * y + 3] << 16) : 0;
}

// one 4x4 block on one wave.  Lane 4m + y (m < 9) predicts row y of mode m from the 13 neighbours
// (held by lanes 0..12, fetched with ds_bpermute) and scores it: the horizontal Hadamard of the
// row in registers, the vertical butterflies across the quad's rows by DPP.  One wave minimum of
// (cost, mode) keys is JM's strict '<' scan in mode order; then dct_luma on lanes 0..15 of the
// chosen prediction (at QP'Y = QPY + QpBdOffsetY)
template <class pel>
__device__ __forceinline__ void i4_block(const DevParams &d, IntraS<pel> &s, MbScratch *scr, int w, int bx4, int by4, const int (&tabr)[2],
                                         bool avL, bool avT, bool avTL, bool avTR, int qpk, int (&acc)[3],
                                         unsigned long long *pst = nullptr) {   // debug: sub-phase stamps [52..57]
#define I4ST(k, v) do { if (pst) { asm volatile("" ::"v"(v)); if (__lane_id() == 0) pst[k] = wall_clock64(); } } while (0)
    I4ST(52, bx4);
    const int lane = threadIdx.x & 63, l = lane & 15;
    const int bx = 4 * bx4, by = 4 * by4, blk = 4 * by4 + bx4;
    const int lambda = d.lambda_mode, qp = d.qp + d.qpbd, had = d.use_hadamard;
    const bool up = by > 0 || avT, left = bx > 0 || avL;
    const bool ul = (bx > 0 && by > 0) || (bx == 0 && by > 0 && avL) || (bx > 0 && by == 0 && avT) || (bx == 0 && by == 0 && avTL);
    bool ur = by == 0 ? (bx + 4 <= 15 ? avT : avTR) : (bx + 4 <= 15);
    if ((bx == 4 || bx == 12) && (by == 4 || by == 12)) ur = false;
    (void)w;
    // P[lane]: p[-1,-1], p[0..7,-1], p[-1,0..3] -- one LDS read per lane from a selected address
    // (the MB's reconstruction or its top / left neighbour samples).  The read is unconditional
    // (an unavailable sample reads rec[0]) and the value selected after it: a load under a
    // condition becomes a divergent branch with its own wait
    // (offsets relative to rec[], selected by masks: nested ?: over lane conditions compile to
    // divergent branches)
    const int mtop = -(int)(lane >= 1 && lane <= 8), mleft = -(int)(lane >= 9);   // else lane 0 (or >= 13)
    const int lx = (lane <= 4 || ur) ? lane - 1 : 3;                               // top row x (lanes 1..8)
    const int px = bx + ((lx & mtop) | (-1 & ~mtop)), py = by + (((lane - 9) & mleft) | (-1 & ~mleft));
    const bool pav = lane < 13 && (lane == 0 ? ul : lane <= 8 ? up : left);
    const int mT = -(int)(py < 0), mL = ~mT & -(int)(px < 0);
    const int ofs = (((int)(s.nb.rtop - s.rec) + px + 1) & mT) | (((int)(s.nb.rleft - s.rec) + py) & mL) | ((16 * py + px) & ~(mT | mL));
    const int raw = s.rec[pav ? ofs : 0];
    const int v = pav ? raw : 0;
    const int upM = by > 0 ? s.ipred_cur[blk - 4] : s.bd.ipm[1 + bx4];
    const int leftM = bx > 0 ? s.ipred_cur[blk - 1] : s.bd.ipm[6 + by4];
    const int mpm = (upM < 0 || leftM < 0) ? 2 : min(upM, leftM);
    const int m = lane >> 2, y = lane & 3;
    int o[4];
    if constexpr (sizeof(pel) == 1) {         // the row's four samples in one dword
        const uint32_t ow = *reinterpret_cast<const uint32_t *>(s.org + (by + y) * 16 + bx);
#pragma unroll
        for (int x = 0; x < 4; x++) o[x] = (int)((ow >> (8 * x)) & 255u);
    } else {
        const uint2 ow = *reinterpret_cast<const uint2 *>(s.org + (by + y) * 16 + bx);
        o[0] = (int)(ow.x & 0xFFFFu); o[1] = (int)(ow.x >> 16); o[2] = (int)(ow.y & 0xFFFFu); o[3] = (int)(ow.y >> 16);
    }
    const int org = s.org[(by + (l >> 2)) * 16 + bx + (l & 3)];   // the TQ lanes' sample
    int st = 0, sl = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) { st += __builtin_amdgcn_readlane(v, 1 + i); sl += __builtin_amdgcn_readlane(v, 9 + i); }
    const int dc = (up && left) ? (st + sl + 4) >> 3 : left ? (sl + 2) >> 2 : up ? (st + 2) >> 2 : (d.maxv + 1) >> 1;
    I4ST(53, mpm);
    int pr[4], dd[4];
#pragma unroll
    for (int x = 0; x < 4; x++) {
        const int e = (int)(((uint32_t)tabr[x >> 1] >> (16 * (x & 1))) & 0xFFFFu), ty = e & 3;
        const int a = __shfl(v, (e >> 2) & 15, 64), b = __shfl(v, (e >> 6) & 15, 64), c = __shfl(v, (e >> 10) & 15, 64);
        // both filters, then a select by masks (a ?: chain here compiles to divergent branches,
        // each waiting for its ds_bpermute results)
        const int f1 = (a + b + 1) >> 1, f2 = (a + 2 * b + c + 2) >> 2;
        const int m1 = -(int)(ty == 1), m2 = -(int)(ty == 2);
        pr[x] = (f1 & m1) | (f2 & m2) | (dc & ~(m1 | m2));
        dd[x] = o[x] - pr[x];
    }
    int t;
    if (had) {
        const int h0 = dd[0] + dd[1], h1 = dd[0] - dd[1], h2 = dd[2] + dd[3], h3 = dd[2] - dd[3];
        int g[4] = {h0 + h2, h1 + h3, h0 - h2, h1 - h3};
#pragma unroll
        for (int x = 0; x < 4; x++) { const int q = dpp<0xB1>(g[x]); g[x] = (y & 1) ? q - g[x] : g[x] + q; }
#pragma unroll
        for (int x = 0; x < 4; x++) { const int q = dpp<0x4E>(g[x]); g[x] = (y & 2) ? q - g[x] : g[x] + q; }
        t = abs(g[0]) + abs(g[1]) + abs(g[2]) + abs(g[3]);
    } else {
        t = abs(dd[0]) + abs(dd[1]) + abs(dd[2]) + abs(dd[3]);
    }
    t += dpp<0xB1>(t);                        // the quad's rows
    t += dpp<0x4E>(t);
    const int sat = had ? t >> 1 : t;
    const bool avm = m == 2 || ((m == 0 || m == 3 || m == 7) && up) || ((m == 1 || m == 8) && left) || (up && left && ul);
    const int cst = (m < 9 && avm) ? (m == mpm ? 0 : 4 * lambda) + sat : BIGCOST;
    const unsigned key = wave_min_u32((y == 0 && cst < BIGCOST) ? ((unsigned)cst << 4) | (unsigned)m : 0xFFFFFFFFu);
    I4ST(54, key);
    const int best = key == 0xFFFFFFFFu ? 0 : (int)(key & 15u), bc = key == 0xFFFFFFFFu ? BIGCOST : (int)(key >> 4);
    // the winner's prediction at TQ lane l (raster 4y' + x'): register x' of lane 4 best + y'
    const int srcl = 4 * best + (l >> 2);
    const int q01 = __shfl((pr[0] & 0xFFFF) | (pr[1] << 16), srcl, 64), q23 = __shfl((pr[2] & 0xFFFF) | (pr[3] << 16), srcl, 64);
    const int qx = (l & 2) ? q23 : q01;
    const int pp = (l & 1) ? (int)((uint32_t)qx >> 16) : (qx & 0xFFFF);
    I4ST(55, pp);
    // dct_luma on every 16-lane group (the four groups compute the same block: no divergent
    // region around the lane exchanges), lanes 0..15 store
    const int c = quad_fwd4x4(org - pp, l);
    int lev, dq, cc;
    unsigned nz = lane_quant(c, l, qp, qpk, false, lev, dq, cc);
    I4ST(56, dq);
    const int rc = quad_inv4x4(dq, l, pp, d.maxv);
    if (lane < 16) {
        scr->i4lev[blk][l] = (int16_t)lev;
        s.rec[(by + (l >> 2)) * 16 + bx + (l & 3)] = (pel)rc;
        if (l == 0) s.ipred_cur[blk] = (int8_t)best;
    }
    nz = __builtin_amdgcn_readlane(nz, 0);
    I4ST(57, nz);
#undef I4ST
    acc[0] += bc;
    if (nz) { acc[1] |= 1 << ((by4 >> 1) * 2 + (bx4 >> 1)); acc[2] |= 1 << blk; }
}

