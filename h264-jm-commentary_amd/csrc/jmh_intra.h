// jmh_intra.h -- intra neighbourhood loads and the Intra16x16 SATD decision shared by the RDO-off
// intra analysis (jmh_analyse.hip) and the RD intra candidates (k_rdo_intra, jmh_rdo.hip).
#pragma once
#include "jmh_common.h"

// Intra4x4 prediction (8.3.1.2) of mode m at pixel l as a formula over P[0..12]
// (P[0] = p[-1,-1], P[1+i] = p[i,-1], P[9+j] = p[-1,j]): type | a << 2 | b << 6 | c << 10,
// type 1: (Pa + Pb + 1) >> 1, 2: (Pa + 2 Pb + Pc + 2) >> 2 (a copy when a == b == c), 3: DC.
static __constant__ uint16_t c_i4tab[9][16] = {
    {0x0446, 0x088A, 0x0CCE, 0x1112, 0x0446, 0x088A, 0x0CCE, 0x1112, 0x0446, 0x088A, 0x0CCE, 0x1112, 0x0446, 0x088A, 0x0CCE, 0x1112},
    {0x2666, 0x2666, 0x2666, 0x2666, 0x2AAA, 0x2AAA, 0x2AAA, 0x2AAA, 0x2EEE, 0x2EEE, 0x2EEE, 0x2EEE, 0x3332, 0x3332, 0x3332, 0x3332},
    {0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003, 0x0003},
    {0x0C86, 0x10CA, 0x150E, 0x1952, 0x10CA, 0x150E, 0x1952, 0x1D96, 0x150E, 0x1952, 0x1D96, 0x21DA, 0x1952, 0x1D96, 0x21DA, 0x221E},
    {0x2406, 0x0842, 0x0C86, 0x10CA, 0x2A42, 0x2406, 0x0842, 0x0C86, 0x2EA6, 0x2A42, 0x2406, 0x0842, 0x32EA, 0x2EA6, 0x2A42, 0x2406},
    {0x0041, 0x0085, 0x00C9, 0x010D, 0x0426, 0x0842, 0x0C86, 0x10CA, 0x026A, 0x0041, 0x0085, 0x00C9, 0x26AE, 0x0426, 0x0842, 0x0C86},
    {0x0241, 0x0426, 0x004A, 0x048E, 0x02A5, 0x2A42, 0x0241, 0x0426, 0x02E9, 0x2EA6, 0x02A5, 0x2A42, 0x032D, 0x32EA, 0x02E9, 0x2EA6},
    {0x0085, 0x00C9, 0x010D, 0x0151, 0x0C86, 0x10CA, 0x150E, 0x1952, 0x00C9, 0x010D, 0x0151, 0x0195, 0x10CA, 0x150E, 0x1952, 0x1D96},
    {0x02A5, 0x2EA6, 0x02E9, 0x32EA, 0x02E9, 0x32EA, 0x032D, 0x332E, 0x032D, 0x332E, 0x3332, 0x3332, 0x3332, 0x3332, 0x3332, 0x3332}};

// intra neighbourhood of an MB in LDS (unfiltered reconstruction of the current picture);
// pel = uint8_t (bit depth 8) or uint16_t (High 10, k_mb_intra only)
template <class pel>
struct IntraNb {
    pel orgc[2][64];
    pel rtop[24];                             // luma row y = -1, x = -1..19 -> [x + 1]
    pel rleft[16];
    pel ctop[2][12];                          // chroma rows y = -1, x = -1..7 -> [x + 1]
    pel cleft[2][8];
};
// prefetch of the intra neighbourhood by threads t in [0, 96)
template <class pel>
__device__ __forceinline__ void load_intra_nb(const DevParams &d, IntraNb<pel> &nb, int t, int mbx, int mby) {
    const pel *recY = spl<pel>(d.recY), *recU = spl<pel>(d.recU), *recV = spl<pel>(d.recV);
    const int pix_x = 16 * mbx, pix_y = 16 * mby, W = d.W, Wc = d.Wc;
    const MbAvail mav = intra_avail(d, mbx, mby);
    const bool avL = mav.L, avT = mav.T, avTL = mav.TL, avTR = mav.TR;
    if (t < 21) {                                  // luma row y = -1, x = -1..19
        const int x = t - 1;
        const bool av = x < 0 ? avTL : x < 16 ? avT : avTR;
        nb.rtop[x + 1] = av ? recY[(pix_y - 1) * W + pix_x + x] : 0;
    } else if (t < 37) {
        const int y = t - 21;
        nb.rleft[y] = avL ? recY[(pix_y + y) * W + pix_x - 1] : 0;
    } else if (t < 55) {                           // chroma rows y = -1, x = -1..7
        const int i = t - 37, uv = i / 9, x = i - 9 * uv - 1;
        const bool av = x < 0 ? avTL : avT;
        nb.ctop[uv][x + 1] = av ? (uv ? recV : recU)[((pix_y >> 1) - 1) * Wc + (pix_x >> 1) + x] : 0;
    } else if (t < 71) {
        const int i = t - 55, uv = i >> 3, y = i & 7;
        nb.cleft[uv][y] = avL ? (uv ? recV : recU)[((pix_y >> 1) + y) * Wc + (pix_x >> 1) - 1] : 0;
    }
}
template <class pel>
__device__ __forceinline__ void load_orgc(const DevParams &d, IntraNb<pel> &nb, int t, int mbx, int mby) {   // t in [0, 128)
    const int uv = t >> 6, k = t & 63;
    nb.orgc[uv][k] = spl<pel>(uv ? d.orgV : d.orgU)[((8 * mby) + (k >> 3)) * d.Wc + 8 * mbx + (k & 7)];
}

// intrapred_luma_16x16 + find_sad_16x16 on one wave (4 modes x 16 blocks = 64 lanes): the
// find_sad_16x16 cost and mode, wave-uniform.  The prediction's parameters (8.3.3: the DC sums and
// the plane's H / V) come from lane reductions -- lanes 0..15 hold p[k, -1], 16..31 p[-1, k]:
// H = sum (k - 7) p[k, -1] - 8 p[-1, -1], V likewise -- and every lane selects its mode's sample
// without branching (a per-lane mode switch ran all four paths on every lane).  The whole wave
// must be active.
template <class pel>
__device__ __forceinline__ void i16_pick(const DevParams &d, const pel *org, const IntraNb<pel> &nb, int lane, bool avL, bool avT, bool avTL,
                                         int &cost16, int &mode16) {
    const int m = lane >> 4, b = lane & 15, ox = (b & 3) * 4, oy = (b >> 2) * 4;
    const pel *T = nb.rtop + 1, *L = nb.rleft;
    const int k = lane & 15, nv = lane < 16 ? (int)T[k] : (int)L[k];
    const int s1 = row16_sum(nv), s2 = row16_sum((k - 7) * nv);
    const int st = __builtin_amdgcn_readlane(s1, 0), sl = __builtin_amdgcn_readlane(s1, 16);
    const int corner = T[-1];
    const int ih = __builtin_amdgcn_readlane(s2, 0) - 8 * corner, iv = __builtin_amdgcn_readlane(s2, 16) - 8 * corner;
    const int dcv = (avT && avL) ? (st + sl + 16) >> 5 : avT ? (st + 8) >> 4 : avL ? (sl + 8) >> 4 : (d.maxv + 1) >> 1;
    const int ib = (5 * ih + 32) >> 6, ic = (5 * iv + 32) >> 6, iaa = 16 * (L[15] + T[15]);
    int tx[4], ly[4];
#pragma unroll
    for (int i = 0; i < 4; i++) { tx[i] = T[ox + i]; ly[i] = L[oy + i]; }
    int mm[16], t[16];
#pragma unroll
    for (int yy = 0; yy < 4; yy++) {
        int o[4];
        if constexpr (sizeof(pel) == 1) {
            const uint32_t w = *reinterpret_cast<const uint32_t *>(org + (oy + yy) * 16 + ox);
#pragma unroll
            for (int xx = 0; xx < 4; xx++) o[xx] = (int)((w >> (8 * xx)) & 255u);
        } else {
#pragma unroll
            for (int xx = 0; xx < 4; xx++) o[xx] = org[(oy + yy) * 16 + ox + xx];
        }
#pragma unroll
        for (int xx = 0; xx < 4; xx++) {
            const int pl = clipmx((iaa + (ox + xx - 7) * ib + (oy + yy - 7) * ic + 16) >> 5, d.maxv);
            const int p = m == 0 ? tx[xx] : m == 1 ? ly[yy] : m == 2 ? dcv : pl;
            mm[4 * yy + xx] = o[xx] - p;
        }
    }
    for (int yy = 0; yy < 4; yy++) {
        int *r = mm + 4 * yy;
        int a0 = r[0] + r[3], a1 = r[1] + r[2], a2 = r[1] - r[2], a3 = r[0] - r[3];
        t[4 * yy] = a0 + a1; t[4 * yy + 2] = a0 - a1; t[4 * yy + 1] = a2 + a3; t[4 * yy + 3] = a3 - a2;
    }
    int acs = 0, dcc = 0;
    for (int xx = 0; xx < 4; xx++) {
        int a0 = t[xx] + t[12 + xx], a1 = t[4 + xx] + t[8 + xx], a2 = t[4 + xx] - t[8 + xx], a3 = t[xx] - t[12 + xx];
        int o0 = a0 + a1, o2 = a0 - a1, o1 = a2 + a3, o3 = a3 - a2;
        if (xx == 0) dcc = o0; else acs += abs(o0);
        acs += abs(o1) + abs(o2) + abs(o3);
    }
    const int cost = row16_sum(acs) + lane_had_abs(dcc / 4, b);
    const bool av16[4] = {avT, avL, true, avT && avL && avTL};
    int best = MAX_VALUE, i16mode = 2;
#pragma unroll
    for (int k2 = 0; k2 < 4; k2++) {
        const int c = __builtin_amdgcn_readlane(cost, 16 * k2);
        if (av16[k2] && c < best) { best = c; i16mode = k2; }
    }
    cost16 = best / 2;
    mode16 = i16mode;
}


// the Intra16x16 DC path of dct_luma_16x16 [J] on one lane: dc[16] (the blocks' DC coefficients,
// raster) -> the 4x4 Hadamard, the DC levels (scan order) in dclev and the dequantised DCs in dcdq
__device__ __forceinline__ void i16_dc(int *dc, int16_t *dclev, int *dcdq, int qp, int qp_const) {
    const int qp_per = qp / 6, qp_rem = qp % 6, q_bits = 15 + qp_per, qp_const2 = qp_const << 1;
    for (int yy = 0; yy < 4; yy++) {
        int *r = dc + 4 * yy;
        int a0 = r[0] + r[3], a3 = r[0] - r[3], a1 = r[1] + r[2], a2 = r[1] - r[2];
        r[0] = a0 + a1; r[2] = a0 - a1; r[1] = a3 + a2; r[3] = a3 - a2;
    }
    for (int xx = 0; xx < 4; xx++) {
        int a0 = dc[xx] + dc[12 + xx], a3 = dc[xx] - dc[12 + xx], a1 = dc[4 + xx] + dc[8 + xx], a2 = dc[4 + xx] - dc[8 + xx];
        dc[xx] = (a0 + a1) >> 1; dc[8 + xx] = (a0 - a1) >> 1; dc[4 + xx] = (a3 + a2) >> 1; dc[12 + xx] = (a3 - a2) >> 1;
    }
    int lev[16];
    for (int k = 0; k < 16; k++) {
        int pos = scan_of(k);
        int level = (abs(dc[pos]) * c_q3[qp_rem][0] + qp_const2) >> (q_bits + 1);
        dclev[k] = (int16_t)isign(level, dc[pos]);
        lev[pos] = dclev[k];
    }
    int t[16];
    for (int yy = 0; yy < 4; yy++) {
        const int *cc = lev + 4 * yy;
        int e0 = cc[0] + cc[2], e1 = cc[0] - cc[2], e2 = cc[1] - cc[3], e3 = cc[1] + cc[3];
        t[4 * yy] = e0 + e3; t[4 * yy + 3] = e0 - e3; t[4 * yy + 1] = e1 + e2; t[4 * yy + 2] = e1 - e2;
    }
    int v00 = c_dq3[qp_rem][0];
    for (int xx = 0; xx < 4; xx++) {
        int e0 = t[xx] + t[8 + xx], e1 = t[xx] - t[8 + xx], e2 = t[4 + xx] - t[12 + xx], e3 = t[4 + xx] + t[12 + xx];
        int fv[4] = {e0 + e3, e1 + e2, e1 - e2, e0 - e3};
        for (int yy = 0; yy < 4; yy++) dcdq[4 * yy + xx] = (fv[yy] * v00 * (1 << qp_per) + 2) >> 2;
    }
}

// dct_luma_16x16 [J] on 256 threads (tid = 16 * blk + l, blk = the 4x4 block in raster order, l =
// the lane's raster position in it): p / org = the lane's prediction and source sample.  Returns
// the lane's AC level (scan position l of block blk; 0 at l == 0) and reconstruction; the DC levels
// (scan order) land in dclev and the per-block AC non-zero flags in bnz (LDS).  dc / dcdq: LDS
// scratch.  Every thread of the workgroup must call it (two barriers).
// act false (wave-uniform: the chroma / idle waves of a 512-thread final): only the barriers.
__device__ __forceinline__ void i16_code(int p, int org, int qp, int qp_const, int *dc, int *dcdq, int16_t *dclev, int *bnz, int tid,
                                         int maxv, int &lev_out, int &rec_out, bool act = true) {
    if (!act) { __syncthreads(); __syncthreads(); lev_out = rec_out = 0; return; }
    const int blk = tid >> 4, l = tid & 15;
    const int c = lane_fwd4x4(org - p, l);
    if (l == 0) dc[blk] = c;
    __syncthreads();
    if (tid == 0) i16_dc(dc, dclev, dcdq, qp, qp_const);
    __syncthreads();
    int lev, dq, cc;
    unsigned nz = lane_quant(c, l, qp, qp_const, true, lev, dq, cc);
    if (l == 0) { dq = dcdq[blk]; bnz[blk] = nz != 0; }
    lev_out = lev;
    rec_out = lane_inv4x4(dq, l, p, maxv);
}
