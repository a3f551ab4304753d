// jmh_rdo.hip — encode_one_macroblock with RDOptimization = 1 [J] on the device (row f4, config 5):
// the rate-distortion loop of rdopt.c (RDCost_for_macroblocks, RDCost_for_8x8blocks,
// RDCost_for_4x4IntraBlocks; with Transform8x8Mode RDCost_for_8x8IntraBlocks and the 8x8 transform per
// inter candidate) with J = SSD + lambda * R and R the CABAC rate of the slice's coding state
// (jmh_cabac_rate.h; the CPU oracle oracle/rdo.c prices the same candidates with its own 9.3.4.2
// coder, and tests/test_rate_xcheck.py compares the two on every candidate).  DESIGN.md §9 has the
// schedule; one tick of the RD stage schedule runs
//   k_rdo_inter   P MBs, one wave each: the EPZS searches, P8x8 block by block (the sub-modes coded a
//                 pass each, rated on four lanes side by side, a wave-uniform decision), the
//                 residual coding of the skip / 16x16 / 16x8 / 8x16 / P8x8 candidates (Transform8x8Mode:
//                 16x16 / 16x8 / 8x16 / all-8x8 P8x8 again with the 8x8 transform) and their chroma;
//   k_rdo_intra   all MBs, one wave each: Intra16x16, the four chroma intra modes, Intra4x4 by
//                 per-block RD (9 modes x 16 lanes code in three passes, 9 lanes rate); Transform8x8Mode:
//                 Intra8x8 by per-block RD (a pass per mode, lane = sample, 9 lanes rate);
//   k_rdo_final   all MBs: one lane per macroblock candidate rates it on its own LDS copy of the
//                 contexts, the strict-'<' minimum of D + lambda R in JM's order wins; results,
//                 reconstruction, the slice's next coding state, the fused DeblockMb.
// Candidates travel to k_rdo_final through the tick's scratch (RdoScr, HBM).  SymbolMode 0: the same
// loop with R the CAVLC bit count (jmh_cavlc_rate.h: nC from the neighbours' and the decided blocks'
// TotalCoeff, the slice's mb_skip_run in place of the coding state; oracle/cavlc_bits.c is its check).
// docs/JM_SEMANTICS.md items 53-60, 63 and 64 pin every RD choice.
#include <type_traits>
#include "jmh_epzs.h"
#include "jmh_intra.h"
#include "jmh_deblock.h"
// Table 9-44 in LDS for every kernel of this file that codes bins (filled by jmr_lds_tables_load)
__shared__ uint32_t g_jmr_lps[64];   // rangeTabLPS[s][0..3] packed per state
__shared__ uint8_t g_jmr_tlps[64];   // transIdxLPS
#if defined(__HIP_DEVICE_COMPILE__)
#define JMR_LPS(s, q) ((g_jmr_lps[s] >> (8 * (q))) & 0xFF)
#define JMR_TLPS(s) g_jmr_tlps[s]
#endif
#include "jmh_cabac_rate.h"
#include "jmh_cavlc_rate.h"

// the LDS tables by threads [0, n); the caller synchronises before the first bin
__device__ __forceinline__ void jmr_lds_tables_load(int t, int n) {
    for (int i = t; i < 64 + 16; i += n) {
        if (i < 64) g_jmr_lps[i] = reinterpret_cast<const uint32_t *>(jmr_lps)[i];
        else reinterpret_cast<uint32_t *>(g_jmr_tlps)[i - 64] = reinterpret_cast<const uint32_t *>(jmr_trans_lps)[i - 64];
    }
}

// luma candidates: 0 P_Skip, 1 16x16, 2 16x8, 3 8x16, 4 P8x8, 5 I16MB, 6 I4MB, 7 I8MB; Transform8x8Mode:
// 8..10 the 16x16 / 16x8 / 8x16 and 11 the (all sub-modes 8x8) P8x8 with the 8x8 transform
#define RD_NL 12
#define RD_NCAND 21   // macroblock-loop candidates: 9 inter + (I16, I4, I8) x 4 chroma modes
__device__ __forceinline__ int rd_cbase(int i) { return i >= 8 ? i - 7 : i; }   // an inter candidate's base / chroma
__device__ __forceinline__ bool rd_t8(int i) { return i >= 7; }                 // luma with the 8x8 transform

// J = D + lambda * R in double, no contraction (the oracle's gcc x86-64 build has none either)
__device__ __forceinline__ double rd_cost(int dist, int bits, double lambda) {
#pragma clang fp contract(off)
    return (double)dist + lambda * (double)bits;
}

// one luma sample at quarter-pel picture position (X, Y) of the MC of a candidate: from the
// searches' LDS window when the whole wave's 6x6 neighbourhoods lie inside it (the window holds the
// UMV-clamped reference, so the values are those of qpel_direct), else from the picture in HBM
template <class pel>
__device__ __forceinline__ int qpel_mb(const DevParams &d, const EpzS<pel> &e, const EWin<pel> &wn, int X, int Y) {
    const int x = X >> 2, y = Y >> 2, wdim = 16 + 2 * min(2 * d.sr + 4, EGeo<pel>::off);
    const bool in = x - 2 >= wn.wx0 && x + 3 < wn.wx0 + EGeo<pel>::ew && y - 2 >= wn.wy0 && y + 3 < wn.wy0 + wdim;
    if (__all(in)) {
        const pel *g = e.g + (size_t)(0 - wn.wy0) * EGeo<pel>::ew - wn.wx0;
        return qpel_from([&](int xx, int yy) { return (int)g[yy * EGeo<pel>::ew + xx]; }, X, Y, d.maxv);
    }
    return qpel_direct(spl<pel>(d.refY), d.W, d.H, X, Y, d.maxv);
}

template <class pel>
struct RdoLuma {                  // one luma candidate
    int16_t luma[16][16];         // levels as jmh_mb_result.luma (I16: AC at [1..15])
    int16_t luma_dc[16];          // I16 DC levels, scan order
    int16_t mv[16][2];            // the MVs per 4x4
    int16_t mvd[16][2];           // mvd of the partition covering each 4x4
    pel rec[256];
    int8_t ipm[16];               // I4: rem_intra4x4_pred_mode (-1: the predicted mode)
    int8_t imode[16];             // I4: the modes
    int8_t b8mode[4];
    int32_t cbp, cbp_blk, dist, i16mode;
};
template <class pel>
struct RdoChroma {                // one chroma candidate (an inter candidate's MC, an intra mode)
    int16_t dc[2][4];
    int16_t ac[2][4][16];
    pel rec[2][64];
    int32_t cbpc, dist;
};
// the CABAC rate of an intra macroblock candidate, coded by k_rdo_intra (beside k_rdo_inter)
struct RdoRate {
    int32_t bits;
    uint32_t range;               // codIRange after it
    jmr_mbinfo out;               // what it leaves for the neighbours' context selection
    int16_t mvw[16][2];           // jmr_mb's work buffer
    alignas(4) uint8_t ctx[JMR_NCTX];   // the contexts after it
};
template <class pel>
struct RdoScr {
    RdoLuma<pel> L[RD_NL];
    RdoChroma<pel> C[9];          // [0..4]: chroma of L[0..4] (and of L[8..11]); [5 + m]: intra chroma mode m
    RdoRate R[12];                // [m]: I16MB with chroma mode m, [4 + m]: I4MB, [8 + m]: I8MB (available modes only)
};
size_t jmh_rdo_scratch_bytes() { return sizeof(RdoScr<uint16_t>); }

// the coding state of the slice at the start of macroblock a into st (LDS, 4-aligned) by threads
// [0, n): initialised (9.3.1.1) at the slice's first macroblock; returns codIRange.  CAVLC (item 64):
// no contexts; returns the slice's mb_skip_run before a
__device__ __forceinline__ uint32_t rdo_state_load(const DevParams &d, int a, uint8_t *st, int t, int n) {
    const int slice = a / d.slice_mbs;
    if (d.cavlc) return a % d.slice_mbs == 0 ? 0 : d.rp->range[slice];
    if (a % d.slice_mbs == 0) {
        for (int i = t; i < JMR_NCTX; i += n) st[i] = jmr_init_one(i, d.slice_type != JMH_P_SLICE, d.qp);
        return 510;
    }
    const uint32_t *src = reinterpret_cast<const uint32_t *>(d.rp->cab + (size_t)slice * JMR_NCTX);
    for (int i = t; i < JMR_NCTX / 4; i += n) reinterpret_cast<uint32_t *>(st)[i] = src[i];
    return d.rp->range[slice];
}
// the neighbours' context-selection records (A left, B above; flags 0 when not available)
__device__ __forceinline__ void rdo_nb_load(const DevParams &d, int mbx, int mby, jmr_mbinfo &A, jmr_mbinfo &B, int &hasA, int &hasB, int t) {
    const MbAvail mav = mb_avail(d, mbx, mby);
    const int a = mby * d.mbw + mbx, nw = (int)sizeof(jmr_mbinfo) / 4;
    if (t < nw) {
        if (mav.L) reinterpret_cast<uint32_t *>(&A)[t] = reinterpret_cast<const uint32_t *>(d.rp->mbi + a - 1)[t];
        if (mav.T) reinterpret_cast<uint32_t *>(&B)[t] = reinterpret_cast<const uint32_t *>(d.rp->mbi + a - d.mbw)[t];
    }
    if (t == 0) { hasA = mav.L; hasB = mav.T; }
}
// ChromaResidualCoding [J] of one candidate on ONE wave, a component per pass (lane = 4x4 block
// cb4 x 16 + l): prediction = intra mode cm (nb) or the MC of fmv; skipped (P_Skip): no residual.
// The 2x2 DC of a component reads its four blocks' DC lanes (wave-uniform).  Writes out (global)
// except its distortion, returned (wave-uniform).
template <class pel>
__device__ __forceinline__ int chroma_cand_w(const DevParams &d, const pel *oc0, const pel *oc1, int ostr, const IntraNb<pel> *nb, int cm, const int16_t (*fmv)[2],
                                             bool skipped, RdoChroma<pel> *out, int lane, int mbx, int mby, bool avT, bool avL) {
    const int maxv = d.maxv, Wc = d.Wc, pix_x = 16 * mbx, pix_y = 16 * mby;
    const int qpi = iclip(-d.qpbd, 51, d.qp + d.cqp_off), qpcy = qpi < 0 ? qpi : c_qpc[qpi], qpc = qpcy + d.qpbd;
    const int cq_bits = 15 + qpc / 6, cqp_const = q_round(d.qsel, cq_bits), qp_per = qpc / 6, qp_rem = qpc % 6;
    const int cb4 = lane >> 4, l = lane & 15;
    const int cxo = (cb4 & 1) * 4 + (l & 3), cyo = (cb4 >> 1) * 4 + (l >> 2);
    int e2 = 0, cr = 0;
#pragma unroll 1
    for (int uv = 0; uv < 2; uv++) {
        int pv;
        if (nb) pv = chroma_pred_px(nb->ctop[uv] + 1, nb->cleft[uv], nb->ctop[uv][0], avT, avL, cm, cxo, cyo, maxv);
        else {   // OneComponentChromaPrediction4x4 [J] / 8.4.2.2.2
            const pel *R = spl<pel>(uv ? d.refV : d.refU);
            const int vx = fmv[(cyo >> 1) * 4 + (cxo >> 1)][0], vy = fmv[(cyo >> 1) * 4 + (cxo >> 1)][1];
            const int ii = ((pix_x >> 1) + cxo) * 8 + vx, jj = ((pix_y >> 1) + cyo) * 8 + vy;
            const int x0 = iclip(0, Wc - 1, ii >> 3), y0 = iclip(0, d.Hc - 1, jj >> 3);
            const int x1 = iclip(0, Wc - 1, (ii + 7) >> 3), y1 = iclip(0, d.Hc - 1, (jj + 7) >> 3);
            const int fx = ii & 7, fy = jj & 7;
            pv = ((8 - fx) * (8 - fy) * R[y0 * Wc + x0] + fx * (8 - fy) * R[y0 * Wc + x1] + (8 - fx) * fy * R[y1 * Wc + x0] +
                  fx * fy * R[y1 * Wc + x1] + 32) >> 6;
        }
        const int org = (uv ? oc1 : oc0)[cyo * ostr + cxo];
        int rv = pv, lev = 0, dcl = 0;
        if (!skipped) {
            const int c = lane_fwd4x4(org - pv, l);
            int cdq, cc;
            const unsigned nz = lane_quant(c, l, qpc, cqp_const, true, lev, cdq, cc);
            int m[4], cost = 0, acany = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                m[q] = __builtin_amdgcn_readlane(c, 16 * q);
                cost += __builtin_amdgcn_readlane(cc, 16 * q);
                acany |= __builtin_amdgcn_readlane((int)nz, 16 * q);
            }
            // the 2x2 DC (dct_chroma), wave-uniform
            const int m1[4] = {m[0] + m[1] + m[2] + m[3], m[0] - m[1] + m[2] - m[3], m[0] + m[1] - m[2] - m[3], m[0] - m[1] - m[2] + m[3]};
            int dcnz = 0, cd[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int level = (abs(m1[k]) * c_q3[qp_rem][0] + 2 * cqp_const) >> (cq_bits + 1);
                if (level) dcnz = 1;
                cd[k] = isign(level, m1[k]);
            }
            const int fv[4] = {cd[0] + cd[1] + cd[2] + cd[3], cd[0] - cd[1] + cd[2] - cd[3], cd[0] + cd[1] - cd[2] - cd[3],
                               cd[0] - cd[1] - cd[2] + cd[3]};
            if (cost < 4) { cdq = 0; lev = 0; }            // _CHROMA_COEFF_COST_
            if (l == 0) cdq = (fv[cb4] * 16 * c_dq3[qp_rem][0] * (1 << qp_per)) >> 5;   // 8.5.11.2
            rv = lane_inv4x4(cdq, l, pv, maxv);
            dcl = cd[l & 3];
            if (dcnz) cr = max(cr, 1);
            if (acany && cost >= 4) cr = 2;
        }
        out->ac[uv][cb4][l] = (int16_t)lev;
        out->rec[uv][cyo * 8 + cxo] = (pel)rv;
        if (lane < 4) out->dc[uv][lane] = (int16_t)dcl;
        e2 += (org - rv) * (org - rv);
    }
    if (lane == 0) out->cbpc = cr;
    return wave_sum(e2);
}

// ======================================================================================
//  role "inter" (k_rdo_inter): ONE WAVE per P macroblock, wave-synchronous LDS (no workgroup
//  barrier): the searches, P8x8 by RDCost_for_8x8blocks, the inter candidates
// ======================================================================================
// an 8x8 block's sub-mode candidates (P8x8 loop): live from the block's last search to its decision,
// so for 16-bit samples they overlay the searches' sub-pel planes (hp, b1: four MBs per CU)
struct RdoP8Tmp {
    alignas(4) uint8_t stc[4][JMR_NCTX];   // per sub-mode rate lane
    int16_t lev8[4][4][16];       // per sub-mode: the 8x8 block's four 4x4 levels (coding order)
    int16_t mvd8[4][4][2];
};
template <class pel>
struct RdoP8Px {
    alignas(4) pel pred8[4][64], rec8[4][64];
};
template <class pel, bool OVERLAY = (sizeof(pel) == 2)>
struct RdoP8Own {
    RdoP8Tmp t;
    RdoP8Px<pel> px;
};
template <class pel>
struct RdoP8Own<pel, true> {};
template <class pel>
struct RdoInterS {
    EpzS<pel> e;                  // the motion searches
    int16_t pmv[8][16][2];        // the MVP each search used (the candidates' mvds)
    alignas(4) uint8_t st0[JMR_NCTX];      // the slice's coding state at the MB start
    alignas(4) uint8_t strun[JMR_NCTX];    // the P8x8 running state (decided 8x8 blocks)
    RdoP8Own<pel> own;
    jmr_mbinfo nbA, nbB;
    jmr_cur currun, curc[4];
    int cost8[4], blk8[4], dist8[4], bits8[4];
    uint32_t rgc[4];
    alignas(4) pel p8pred[256], p8rec[256];   // the P8x8 candidate, assembled block by block
    int16_t p8lev[16][16];
    int16_t fmv[16][2];           // MVs of the candidate being coded
    int16_t bcost[16];            // per 4x4: coefficient cost (saturated at 32767: MAX_VALUE for a level > 1), non-zero levels
    uint8_t bnz[16];
};

// LumaResidualCoding [J] of an inter candidate (4x4 transform) on one wave, a row of 4x4 blocks per
// pass: MC of s.fmv, LumaResidualCoding8x8's _LUMA_COEFF_COST_ zeroing and the macroblock one;
// skipped: prediction only
template <class pel>
__device__ __forceinline__ void luma_inter(const DevParams &d, RdoInterS<pel> &s, const EWin<pel> &wn, RdoLuma<pel> *L, bool skipped, int mbx, int mby,
                                           int lane) {
    const int l = lane & 15, qp = d.qp + d.qpbd, maxv = d.maxv, rnd = q_round(d.qsel, 15 + qp / 6);
    int lev[4], rv[4], pr[4], org[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int blk = 4 * i + (lane >> 4), px4 = 4 * (blk & 3) + (l & 3), py4 = 4 * i + (l >> 2);
        pr[i] = qpel_mb(d, s.e, wn, 4 * (16 * mbx + px4) + s.fmv[blk][0], 4 * (16 * mby + py4) + s.fmv[blk][1]);
        org[i] = s.e.org[py4 * 16 + px4];
        lev[i] = 0; rv[i] = pr[i];
        if (!skipped) {
            const int c = lane_fwd4x4(org[i] - pr[i], l);
            int dq, cc;
            const unsigned nz = lane_quant(c, l, qp, rnd, false, lev[i], dq, cc);
            rv[i] = lane_inv4x4(dq, l, pr[i], maxv);
            if (l == 0) { s.bcost[blk] = (int16_t)min(cc, 32767); s.bnz[blk] = nz != 0; }   // saturated: only its sums are compared (with 4 and 5)
        }
    }
    int cbp = 0, cbp_blk = 0;
    if (!skipped) {
        wave_lds_sync();
        int sum_cnt = 0, keep8 = 0;
        for (int b8 = 0; b8 < 4; b8++) {                // wave-uniform
            const int base = (b8 >> 1) * 8 + (b8 & 1) * 2;
            int c8 = s.bcost[base] + s.bcost[base + 1] + s.bcost[base + 4] + s.bcost[base + 5];
            const int nz8 = s.bnz[base] | s.bnz[base + 1] | s.bnz[base + 4] | s.bnz[base + 5];
            if (c8 <= 4) c8 = 0;                         // _LUMA_COEFF_COST_
            else {
                keep8 |= 1 << b8;
                if (nz8) cbp |= 1 << b8;
                for (int q = 0; q < 4; q++) {
                    const int k = base + (q & 1) + (q >> 1) * 4;
                    if (s.bnz[k]) cbp_blk |= 1 << k;
                }
            }
            sum_cnt += c8;
        }
        if (sum_cnt <= 5) { keep8 = 0; cbp = 0; cbp_blk = 0; }   // _LUMA_MB_COEFF_COST_
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int blk = 4 * i + (lane >> 4);
            if (!((keep8 >> (((blk >> 3) << 1) + ((blk & 3) >> 1))) & 1)) { lev[i] = 0; rv[i] = pr[i]; }
        }
    }
    int e2 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int blk = 4 * i + (lane >> 4), px4 = 4 * (blk & 3) + (l & 3), py4 = 4 * i + (l >> 2);
        L->luma[blk][l] = (int16_t)lev[i];
        L->rec[py4 * 16 + px4] = (pel)rv[i];
        e2 += (org[i] - rv[i]) * (org[i] - rv[i]);
    }
    const int dist = wave_sum(e2);
    if (lane == 0) { L->cbp = cbp; L->cbp_blk = cbp_blk; L->dist = dist; L->i16mode = 0; }
}

// LumaResidualCoding [J] of an inter candidate with transform_size_8x8_flag 1 (Transform8x8Mode,
// item 63) on one wave, an 8x8 block per pass (lane = sample): MC of s.fmv, dct_luma8x8 (levels in
// jmh_mb_result's CAVLC interleave), the same _LUMA_COEFF_COST_ zeroing per 8x8 block and per
// macroblock.  The P8x8 assembly buffers (p8pred / p8rec / p8lev, cost8 / blk8) are free by now.
template <class pel>
__device__ __forceinline__ void luma_inter8(const DevParams &d, RdoInterS<pel> &s, const EWin<pel> &wn, RdoLuma<pel> *L, int mbx, int mby,
                                            int lane) {
    const int qp = d.qp + d.qpbd, maxv = d.maxv, rnd = q_round(d.qsel, 16 + qp / 6), x = lane & 7, y = lane >> 3;
#pragma unroll 1
    for (int b8 = 0; b8 < 4; b8++) {
        const int px = 8 * (b8 & 1) + x, py = 8 * (b8 >> 1) + y, k = (py >> 2) * 4 + (px >> 2);
        const int p = qpel_mb(d, s.e, wn, 4 * (16 * mbx + px) + s.fmv[k][0], 4 * (16 * mby + py) + s.fmv[k][1]);
        const int c = wave_fwd8x8((int)s.e.org[py * 16 + px] - p, lane);
        int lev, dq, cost;
        const unsigned long long nz = wave_quant8(c, lane, qp, rnd, lev, dq, cost);
        s.p8pred[py * 16 + px] = (pel)p;
        s.p8rec[py * 16 + px] = (pel)wave_inv8x8(dq, lane, p, maxv);
        s.p8lev[il_blk(b8, lane)][lane >> 2] = (int16_t)lev;
        if (lane == 0) { s.cost8[b8] = cost; s.blk8[b8] = nz != 0; }
    }
    wave_lds_sync();
    int sum = 0, keep = 0, cbp = 0, cbp_blk = 0;        // wave-uniform
    for (int b8 = 0; b8 < 4; b8++) {
        const int c8 = s.cost8[b8] <= 4 ? 0 : s.cost8[b8];   // _LUMA_COEFF_COST_
        if (c8) {
            keep |= 1 << b8;
            if (s.blk8[b8]) { cbp |= 1 << b8; cbp_blk |= 0x33 << ((b8 >> 1) * 8 + (b8 & 1) * 2); }
        }
        sum += c8;
    }
    if (sum <= 5) keep = cbp = cbp_blk = 0;             // _LUMA_MB_COEFF_COST_
    int e2 = 0;
    for (int i = lane; i < 256; i += 64) {
        const int b8 = ((i >> 7) << 1) + ((i & 15) >> 3), kb = (keep >> b8) & 1;
        const pel rv = kb ? s.p8rec[i] : s.p8pred[i];
        L->rec[i] = rv;
        L->luma[i >> 4][i & 15] = ((keep >> (((i >> 7) << 1) + ((i >> 4 & 3) >> 1))) & 1) ? s.p8lev[i >> 4][i & 15] : 0;
        const int e = (int)s.e.org[i] - (int)rv;
        e2 += e * e;
    }
    const int dist = wave_sum(e2);
    if (lane == 0) { L->cbp = cbp; L->cbp_blk = cbp_blk; L->dist = dist; L->i16mode = 0; }
}

// FFS: SearchMode 0 with the MB's SAD tables in ftab (its own instantiation: the table build's
// registers stay out of the EPZS kernel's allocation)
template <class pel, bool T8, bool FFS>
__device__ __forceinline__ void rdo_inter_mb(const DevParams &d, RdoInterS<pel> &s, RdoScr<pel> *scr, uint8_t *ftab_, int mbx, int mby, int lane) {
    uint8_t *const ftab = FFS ? ftab_ : nullptr;
    const int a = mby * d.mbw + mbx, pix_x = 16 * mbx, pix_y = 16 * mby, qp = d.qp + d.qpbd, maxv = d.maxv;
    const MbAvail mav = mb_avail(d, mbx, mby);
    const bool prof = d.prof && lane == 0 && d.prof_mb == a;   // debug (JMH_PHASE_PROF): stamps 40..52
    PSTAMP(40);
    RdoP8Tmp *tp;
    RdoP8Px<pel> *px8;
    if constexpr (sizeof(pel) == 2) {
        static_assert(sizeof(RdoP8Tmp) <= sizeof(s.e.hp) && sizeof(RdoP8Px<pel>) <= sizeof(s.e.b1), "P8x8 overlay");
        tp = reinterpret_cast<RdoP8Tmp *>(&s.e.hp[0][0]);
        px8 = reinterpret_cast<RdoP8Px<pel> *>(&s.e.b1[0][0]);
    } else {
        tp = &s.own.t;
        px8 = &s.own.px;
    }
    // ---- inputs: the searches' window, chroma, the coding state, the neighbours' records
    const EWin<pel> wn = epzs_load_mb(d, s.e, mbx, mby, lane);
    jmr_lds_tables_load(lane, 64);
    int hasA = 0, hasB = 0;
    const uint32_t rg0 = rdo_state_load(d, a, s.st0, lane, 64);
    {
        const int nw = (int)sizeof(jmr_mbinfo) / 4;
        hasA = mav.L; hasB = mav.T;
        if (lane < nw) {
            if (hasA) reinterpret_cast<uint32_t *>(&s.nbA)[lane] = reinterpret_cast<const uint32_t *>(d.rp->mbi + a - 1)[lane];
            if (hasB) reinterpret_cast<uint32_t *>(&s.nbB)[lane] = reinterpret_cast<const uint32_t *>(d.rp->mbi + a - d.mbw)[lane];
        }
    }
    wave_lds_sync();
    PSTAMP(41);
    const jmr_mbinfo *A = hasA ? &s.nbA : nullptr, *B = hasB ? &s.nbB : nullptr;
    // SearchMode 0: the SAD tables of the 41 searches (SetupFastFullPelSearch [J]) around the FFS
    // centre, before the first
    int fcx = 0, fcy = 0;
    if (ftab) {
        int pmx, pmy;
        MvpNb nb;
        set_mvp_nb(NbEpz<EpzS<pel>>{s.e, 1, 0, 0}, 0, 0, 16, 16, pmx, pmy, nb);
        fcx = __builtin_amdgcn_readfirstlane(iclip(-d.sr, d.sr, pmx / 4));
        fcy = __builtin_amdgcn_readfirstlane(iclip(-d.sr, d.sr, pmy / 4));
        ffs_table_build(d, s.e, wn, ftab, fcx, fcy, lane);
        PSTAMP(20);
    }
    // SearchMode 0 with equal ranges: the full-pel argmins of the searches whose MVPs need no other
    // search of their group in one pass over the table phase (ffs_group_min)
    const bool grp = ftab && d.restrict_sr != 0;
    auto mvp = [&](int bt, int bx4, int by4, int bsx, int bsy, int b8, int b88, int &px, int &py) {
        MvpNb nb;
        set_mvp_nb(NbEpz<EpzS<pel>>{s.e, bt, b8, b88}, bx4, by4, bsx, bsy, px, py, nb);
        px = __builtin_amdgcn_readfirstlane(px);
        py = __builtin_amdgcn_readfirstlane(py);
    };
    unsigned gk[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    if (grp) {
        int px[4] = {0, 0, 0, 0}, py[4] = {0, 0, 0, 0};
        mvp(1, 0, 0, 16, 16, 0, 0, px[0], py[0]);
        mvp(2, 0, 0, 16, 8, 0, 0, px[1], py[1]);
        mvp(3, 0, 0, 8, 16, 0, 0, px[2], py[2]);
        ffs_group_min<3>(d, ftab, 0, d.sr, fcx, fcy, px, py, lane, gk);
    }
    // ---- motion estimation for 16x16, 16x8, 8x16 (PartitionMotionSearch [J])
    if constexpr (FFS) {
        // the partitions' first searches, then their second ones (a full search's MVP reads only its
        // own type's earlier results, so the order across types changes nothing)
        epzs_block<1, pel, EPZS_FB_ROWS>(d, s.e, wn, 0, 0, 0, 0, 0, false, s.pmv, ftab, gk[0]);
        epzs_block<2, pel, EPZS_FB_ROWS>(d, s.e, wn, 0, 0, 0, 0, 0, false, s.pmv, ftab, gk[1]);
        epzs_block<3, pel, EPZS_FB_ROWS>(d, s.e, wn, 0, 0, 0, 0, 0, false, s.pmv, ftab, gk[2]);
        if (grp) {
            int px[4] = {0, 0, 0, 0}, py[4] = {0, 0, 0, 0};
            mvp(2, 0, 2, 16, 8, 0, 0, px[0], py[0]);
            mvp(3, 2, 0, 8, 16, 0, 0, px[1], py[1]);
            ffs_group_min<2, 1>(d, ftab, 0, d.sr, fcx, fcy, px, py, lane, gk);
        }
        epzs_block<2, pel, EPZS_FB_ROWS>(d, s.e, wn, 0, 2, 1, 0, 0, false, s.pmv, ftab, gk[0]);
        epzs_block<3, pel, EPZS_FB_ROWS>(d, s.e, wn, 2, 0, 1, 0, 0, false, s.pmv, ftab, gk[1]);
    } else {
        epzs_block<1, pel, EPZS_FB_ROWS>(d, s.e, wn, 0, 0, 0, 0, 0, false, s.pmv, ftab);
        epzs_block<2, pel, EPZS_FB_ROWS>(d, s.e, wn, 0, 0, 0, 0, 0, false, s.pmv, ftab);
        epzs_block<2, pel, EPZS_FB_ROWS>(d, s.e, wn, 0, 2, 1, 0, 0, false, s.pmv, ftab);
        epzs_block<3, pel, EPZS_FB_ROWS>(d, s.e, wn, 0, 0, 0, 0, 0, false, s.pmv, ftab);
        epzs_block<3, pel, EPZS_FB_ROWS>(d, s.e, wn, 2, 0, 1, 0, 0, false, s.pmv, ftab);
    }
    PSTAMP(42);
    const bool p8 = inter_on(d.isr, 4) || inter_on(d.isr, 5) || inter_on(d.isr, 6) || inter_on(d.isr, 7);
    for (int i = lane; i < JMR_NCTX / 4; i += 64) reinterpret_cast<uint32_t *>(s.strun)[i] = reinterpret_cast<const uint32_t *>(s.st0)[i];
    if (lane == 0) memset(&s.currun, 0, sizeof(s.currun));
    uint32_t rgrun = rg0;
    int best8x8 = 0, p8cbp = 0, p8blk = 0, p8cnt = 0;
    wave_lds_sync();
    // ---- P8x8: per 8x8 block the sub-modes' searches, their LumaResidualCoding8x8 (a pass per
    //      sub-mode: four 4x4 blocks x 16 lanes), their RDCost_for_8x8blocks rates (lanes 0, 16,
    //      32, 48 side by side), the decision
    const int b4 = lane >> 4, l = lane & 15;
#pragma unroll 1
    for (int b8 = 0; b8 < 4 && p8; b8++) {
        const int X = 2 * (b8 & 1), Y = 2 * (b8 >> 1);
        if constexpr (FFS) {
        unsigned bk[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        if (grp) {                                      // 8x8, 8x4 top, 4x8 left, 4x4 #0
            int px[4], py[4];
            mvp(4, X, Y, 8, 8, b8, best8x8, px[0], py[0]);
            mvp(5, X, Y, 8, 4, b8, best8x8, px[1], py[1]);
            mvp(6, X, Y, 4, 8, b8, best8x8, px[2], py[2]);
            mvp(7, X, Y, 4, 4, b8, best8x8, px[3], py[3]);
            ffs_group_min<4>(d, ftab, 1 + b8, d.sr, fcx, fcy, px, py, lane, bk);
        }
        epzs_block<4, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y, b8, b8, best8x8, false, s.pmv, ftab, bk[0]);
        epzs_block<5, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y, b8, b8, best8x8, false, s.pmv, ftab, bk[1]);
        epzs_block<6, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y, b8, b8, best8x8, false, s.pmv, ftab, bk[2]);
        epzs_block<7, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y, b8, b8, best8x8, false, s.pmv, ftab, bk[3]);
        if (grp) {                                      // 8x4 bottom, 4x8 right, 4x4 #1
            int px[4] = {0, 0, 0, 0}, py[4] = {0, 0, 0, 0};
            mvp(5, X, Y + 1, 8, 4, b8, best8x8, px[0], py[0]);
            mvp(6, X + 1, Y, 4, 8, b8, best8x8, px[1], py[1]);
            mvp(7, X + 1, Y, 4, 4, b8, best8x8, px[2], py[2]);
            ffs_group_min<3, 1>(d, ftab, 1 + b8, d.sr, fcx, fcy, px, py, lane, bk);
        }
        epzs_block<5, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y + 1, b8, b8, best8x8, false, s.pmv, ftab, bk[0]);
        epzs_block<6, pel, EPZS_FB_ROWS>(d, s.e, wn, X + 1, Y, b8, b8, best8x8, false, s.pmv, ftab, bk[1]);
        epzs_block<7, pel, EPZS_FB_ROWS>(d, s.e, wn, X + 1, Y, b8, b8, best8x8, false, s.pmv, ftab, bk[2]);
        epzs_block<7, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y + 1, b8, b8, best8x8, false, s.pmv, ftab);
        epzs_block<7, pel, EPZS_FB_ROWS>(d, s.e, wn, X + 1, Y + 1, b8, b8, best8x8, false, s.pmv, ftab);
        } else {
        epzs_block<4, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y, b8, b8, best8x8, false, s.pmv, ftab);
        epzs_block<5, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y, b8, b8, best8x8, false, s.pmv, ftab);
        epzs_block<5, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y + 1, b8, b8, best8x8, false, s.pmv, ftab);
        epzs_block<6, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y, b8, b8, best8x8, false, s.pmv, ftab);
        epzs_block<6, pel, EPZS_FB_ROWS>(d, s.e, wn, X + 1, Y, b8, b8, best8x8, false, s.pmv, ftab);
        epzs_block<7, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y, b8, b8, best8x8, false, s.pmv, ftab);
        epzs_block<7, pel, EPZS_FB_ROWS>(d, s.e, wn, X + 1, Y, b8, b8, best8x8, false, s.pmv, ftab);
        epzs_block<7, pel, EPZS_FB_ROWS>(d, s.e, wn, X, Y + 1, b8, b8, best8x8, false, s.pmv, ftab);
        epzs_block<7, pel, EPZS_FB_ROWS>(d, s.e, wn, X + 1, Y + 1, b8, b8, best8x8, false, s.pmv, ftab);
        }
        PSTAMP(43 + 2 * b8);
        const int bx4 = X + (b4 & 1), by4 = Y + (b4 >> 1), k = by4 * 4 + bx4;
        const int px = 4 * bx4 + (l & 3), py = 4 * by4 + (l >> 2), q8 = (4 * (b4 >> 1) + (l >> 2)) * 8 + 4 * (b4 & 1) + (l & 3);
        const int org = s.e.org[py * 16 + px];
#pragma unroll 1
        for (int w = 0; w < 4; w++) {
            const int sm = 4 + w;
            if (!inter_on(d.isr, sm)) continue;         // wave-uniform
            const int p = qpel_mb(d, s.e, wn, 4 * (pix_x + px) + s.e.all_mv[sm][k][0], 4 * (pix_y + py) + s.e.all_mv[sm][k][1]);
            const int c = lane_fwd4x4(org - p, l);
            int lev, dq, cc;
            const unsigned nz = lane_quant(c, l, qp, q_round(d.qsel, 15 + qp / 6), false, lev, dq, cc);
            int rv = lane_inv4x4(dq, l, p, maxv);
            int cost = 0, blk = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                cost += __builtin_amdgcn_readlane(cc, 16 * q);
                const int kq = (Y + (q >> 1)) * 4 + X + (q & 1);
                if (__builtin_amdgcn_readlane((int)nz, 16 * q)) blk |= 1 << kq;
            }
            if (cost <= 4) { cost = 0; blk = 0; lev = 0; rv = p; }   // _LUMA_COEFF_COST_
            tp->lev8[w][b4][l] = (int16_t)lev;
            px8->pred8[w][q8] = (pel)p;
            px8->rec8[w][q8] = (pel)rv;
            const int dist = wave_sum((org - rv) * (org - rv));
            if (lane == 0) { s.cost8[w] = cost; s.blk8[w] = blk; s.dist8[w] = dist; }
            if (lane < 4) {
                const int kk = (Y + (lane >> 1)) * 4 + X + (lane & 1);
                tp->mvd8[w][lane][0] = (int16_t)(s.e.all_mv[sm][kk][0] - s.pmv[sm][kk][0]);
                tp->mvd8[w][lane][1] = (int16_t)(s.e.all_mv[sm][kk][1] - s.pmv[sm][kk][1]);
            }
        }
        if (!d.cavlc)
            for (int i = lane; i < JMR_NCTX; i += 64) {   // each rate lane's copy of the running state
                const int w = i / (JMR_NCTX / 4), j = i % (JMR_NCTX / 4);
                reinterpret_cast<uint32_t *>(tp->stc[w])[j] = reinterpret_cast<const uint32_t *>(s.strun)[j];
            }
        wave_lds_sync();
        if (l == 0 && inter_on(d.isr, 4 + b4)) {        // RDCost_for_8x8blocks' rate, sub-mode 4 + b4
            const int w = b4;
            s.curc[w] = s.currun;
            if (d.cavlc)                                // the decided blocks' TotalCoeff (nC)
                s.bits8[w] = jmv_b8(A, B, &s.curc[w], b8, 4 + w, (const int16_t(*)[2])tp->mvd8[w], s.cost8[w] > 0,
                                    (const int16_t(*)[16])tp->lev8[w]);
            else {
                jmr_eng e = {tp->stc[w], rgrun, 0};
                jmr_b8(&e, A, B, &s.curc[w], b8, 4 + w, (const int16_t(*)[2])tp->mvd8[w], s.cost8[w] > 0, (const int16_t(*)[16])tp->lev8[w]);
                s.bits8[w] = e.bits;
                s.rgc[w] = e.range;
            }
        }
        wave_lds_sync();
        double best = 1e30;                             // wave-uniform decision
        int bm = 0;
        for (int w = 0; w < 4; w++)
            if (inter_on(d.isr, 4 + w)) {
                const double rd = rd_cost(s.dist8[w], s.bits8[w], d.lambda_rd);
                if (rd < best) { best = rd; bm = w; }
            }
        best8x8 |= (4 + bm) << (4 * b8);
        if (!d.cavlc) rgrun = s.rgc[bm];
        if (s.cost8[bm]) { p8cbp |= 1 << b8; p8blk |= s.blk8[bm]; p8cnt += s.cost8[bm]; }
        if (!d.cavlc && lane < JMR_NCTX / 4) reinterpret_cast<uint32_t *>(s.strun)[lane] = reinterpret_cast<const uint32_t *>(tp->stc[bm])[lane];
        if (lane < (int)sizeof(jmr_cur) / 4) reinterpret_cast<uint32_t *>(&s.currun)[lane] = reinterpret_cast<const uint32_t *>(&s.curc[bm])[lane];
        {                                               // the decided block into the P8x8 candidate
            const int yy = lane >> 3, xx = lane & 7;
            s.p8pred[(8 * (b8 >> 1) + yy) * 16 + 8 * (b8 & 1) + xx] = px8->pred8[bm][lane];
            s.p8rec[(8 * (b8 >> 1) + yy) * 16 + 8 * (b8 & 1) + xx] = px8->rec8[bm][lane];
            const int qb = lane >> 4, kk = (Y + (qb >> 1)) * 4 + X + (qb & 1);
            s.p8lev[kk][lane & 15] = tp->lev8[bm][qb][lane & 15];
        }
        wave_lds_sync();
        PSTAMP(44 + 2 * b8);
    }
    RdoLuma<pel> *L = scr->L;
    if (p8) {                                           // SetCoeffAndReconstruction8x8
        const bool zero = p8cnt <= 5;                   // _LUMA_MB_COEFF_COST_
        int e2 = 0;
        for (int i = lane; i < 256; i += 64) {
            const pel rv = zero ? s.p8pred[i] : s.p8rec[i];
            L[4].rec[i] = rv;
            L[4].luma[i >> 4][i & 15] = zero ? 0 : s.p8lev[i >> 4][i & 15];
            const int e = (int)s.e.org[i] - (int)rv;
            e2 += e * e;
        }
        if (lane < 32) {
            const int kk = lane >> 1, c = lane & 1, smk = (best8x8 >> (4 * (((kk >> 3) << 1) + ((kk & 3) >> 1)))) & 15;
            L[4].mv[kk][c] = s.e.all_mv[smk][kk][c];
            L[4].mvd[kk][c] = (int16_t)(s.e.all_mv[smk][kk][c] - s.pmv[smk][kk][c]);
        }
        if (lane < 4) L[4].b8mode[lane] = (int8_t)((best8x8 >> (4 * lane)) & 15);
        const int dist = wave_sum(e2);
        if (lane == 0) { L[4].cbp = zero ? 0 : p8cbp; L[4].cbp_blk = zero ? 0 : p8blk; L[4].dist = dist; L[4].i16mode = 0; }
    }
    // ---- FindSkipModeMotionVector [J] (wave-uniform), the spatial memory of the next MB (its EPZS
    //      predictor 34)
    int skipx, skipy;
    {
        int pcx, pcy;
        set_mvp(NbBorder{s.e.bd}, 0, 0, 16, 16, pcx, pcy);
        NbBorder nbv{s.e.bd};
        int ra = -1, ax = 0, ay = 0, rb = -1, bx = 0, by = 0;
        const bool aa = nbv(-1, 0, ra, ax, ay), ab = nbv(0, -1, rb, bx, by);
        const bool zl = !aa || (ra == 0 && ax == 0 && ay == 0), za = !ab || (rb == 0 && bx == 0 && by == 0);
        skipx = (za || zl) ? 0 : pcx;
        skipy = (za || zl) ? 0 : pcy;
    }
    MbScratch *ms = d.scr + a;
    if (d.epzs_maxts)                                   // item 61: the full-pel costs for the neighbours
        for (int i = lane; i < 7 * 16; i += 64) ms->fpc[i >> 4][i & 15] = s.e.fpc[i >> 4][i & 15];
    for (int i = lane; i < 7 * 32; i += 64) {
        const int m = 1 + i / 32, k = (i & 31) >> 1, c = i & 1;
        ms->all_mv[m][k][c] = s.e.all_mv[m][k][c];
    }
    // ---- the skip / 16x16 / 16x8 / 8x16 candidates (LumaResidualCoding) and the chroma of all five
    //      (ChromaResidualCoding [J], the MC of each candidate's MVs)
#pragma unroll 1
    for (int c = 0; c < 5; c++) {
        if (c == 4 ? !p8 : c > 0 && !inter_on(d.isr, c)) continue;   // uniform
        if (lane < 32) {
            const int k = lane >> 1, cc = lane & 1;
            const int smk = (best8x8 >> (4 * (((k >> 3) << 1) + ((k & 3) >> 1)))) & 15;
            const int v = c == 0 ? (cc ? skipy : skipx) : s.e.all_mv[c == 4 ? smk : c][k][cc];
            s.fmv[k][cc] = (int16_t)v;
            if (c < 4) {
                L[c].mv[k][cc] = (int16_t)v;
                L[c].mvd[k][cc] = (int16_t)(c == 0 ? 0 : v - s.pmv[c][k][cc]);
            }
        }
        if (c < 4 && lane < 4) L[c].b8mode[lane] = (int8_t)c;
        wave_lds_sync();
        if (c < 4) luma_inter(d, s, wn, &L[c], c == 0, mbx, mby, lane);
        // the MB's chroma source straight from the picture (each sample read once per candidate;
        // 128-256 B less LDS, profiles/r7n_rdo_lds_ab.txt)
        const int ostr = d.Wc;
        const pel *oc0 = spl<pel>(d.orgU) + 8 * mby * ostr + 8 * mbx, *oc1 = spl<pel>(d.orgV) + 8 * mby * ostr + 8 * mbx;
        const int dist = chroma_cand_w<pel>(d, oc0, oc1, ostr, nullptr, 0, s.fmv, c == 0, &scr->C[c], lane, mbx, mby, mav.T, mav.L);
        if (lane == 0) scr->C[c].dist = dist;
        wave_lds_sync();
    }
    // ---- Transform8x8Mode (item 63): the same motion with the 8x8 transform: 16x16 / 16x8 / 8x16 and
    //      the P8x8 whose four blocks chose the 8x8 sub-mode; the chroma is the base candidate's
    if constexpr (T8) {
#pragma unroll 1
        for (int c = 1; c <= 4; c++) {
            if (c == 4 ? !(p8 && best8x8 == 0x4444) : !inter_on(d.isr, c)) continue;   // uniform
            if (lane < 32) {
                const int k = lane >> 1, cc = lane & 1, sm = c == 4 ? 4 : c;
                const int v = s.e.all_mv[sm][k][cc];
                s.fmv[k][cc] = (int16_t)v;
                L[c + 7].mv[k][cc] = (int16_t)v;
                L[c + 7].mvd[k][cc] = (int16_t)(v - s.pmv[sm][k][cc]);
            }
            if (lane < 4) L[c + 7].b8mode[lane] = (int8_t)(c == 4 ? 4 : c);
            wave_lds_sync();
            luma_inter8(d, s, wn, &L[c + 7], mbx, mby, lane);
            wave_lds_sync();
        }
    }
    PSTAMP(52);
}

// ======================================================================================
//  role "intra" (k_rdo_intra): ONE WAVE per macroblock, wave-synchronous: Intra16x16, the chroma
//  intra modes, Intra4x4 by RDCost_for_4x4IntraBlocks
// ======================================================================================
// the Intra8x8 decision's state (Transform8x8Mode only: the RDO-off-transform build keeps k_rdo_intra's LDS)
template <class pel, bool T8>
struct RdoI8S {
    alignas(4) pel rec8[256];     // the Intra8x8 reconstruction in progress
    int raw[25], av[25], f[25];   // the reference edge: [7 - y] left, [8] corner, [9 + x] top (8.3.2.2.1)
    int16_t lev8[9][64];          // per mode: levels in 8x8 zig-zag order
    alignas(4) pel r8[9][64];     // per mode: the block's reconstruction (raster)
    int m8[4];                    // the decided modes
};
template <class pel>
struct RdoI8S<pel, false> {};
template <class pel, bool T8>
struct RdoIntraS {
    alignas(4) pel org[256];
    alignas(4) pel rec[256];      // the Intra4x4 reconstruction in progress
    IntraNb<pel> nb;
    Border bd;
    int8_t ipred_cur[16];
    alignas(4) uint8_t st0[JMR_NCTX];
    alignas(4) uint8_t stc[T8 ? 12 : 9][JMR_NCTX];
    RdoI8S<pel, T8> i8;
    jmr_mbinfo nbA, nbB;
    uint8_t tcd[24];              // CAVLC: the TotalCoeff of the blocks decided so far (nC, item 64)
    uint8_t tcm[9][4];            //   ... of each mode's block (Intra4x4: [m][0]; Intra8x8: its four 4x4)
    int P[13];
    int16_t lev[9][16];
    pel r4[9][16];
    int dist[9], bits[9], nz[9];
    int dc[16], dcdq[16];
    int16_t dclev[16];
};

template <class pel, bool T8>
__device__ __forceinline__ int i4_lpix(const RdoIntraS<pel, T8> &s, int x, int y) {
    if (y < 0) return s.nb.rtop[x + 1];
    if (x < 0) return s.nb.rleft[y];
    return s.rec[16 * y + x];
}

// Intra8x8 (Transform8x8Mode, item 63): Mode_Decision_for_8x8IntraBlocks [J] by RDCost_for_8x8IntraBlocks,
// the four blocks in order on one wave: the filtered reference edge (8.3.2.2.1), a pass per mode
// (lane = sample: prediction, dct_luma8x8, reconstruction, SSD), lane m rates mode m from the
// macroblock-start state, a wave-uniform strict-'<' decision; the winner reconstructs
template <class pel, bool CAV>
__device__ __forceinline__ void rdo_intra8(const DevParams &d, RdoIntraS<pel, true> &s, RdoLuma<pel> &L, const jmr_mbinfo *A, const jmr_mbinfo *B,
                                           uint32_t rg0, const MbAvail &mav, int mbx, int mby, int lane) {
    RdoI8S<pel, true> &q = s.i8;
    const int qp = d.qp + d.qpbd, maxv = d.maxv, rnd = q_round(d.qsel, 16 + qp / 6), W = d.W, pix_x = 16 * mbx, pix_y = 16 * mby;
    const int x = lane & 7, y = lane >> 3;
    const pel *recY = spl<pel>(d.recY);
    int cbp = 0, blkm = 0;
#pragma unroll 1
    for (int b8 = 0; b8 < 4; b8++) {
        const int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
        const bool left = bx ? true : mav.L, up = by ? true : mav.T;
        const bool ul = bx && by ? true : bx ? mav.T : by ? mav.L : mav.TL;
        const bool ur = b8 == 0 ? mav.T : b8 == 1 ? mav.TR : b8 == 2;
        if (lane < 25) {
            int xm, ym;
            bool av;
            if (lane < 8) { xm = bx - 1; ym = by + 7 - lane; av = left; }
            else if (lane == 8) { xm = bx - 1; ym = by - 1; av = ul; }
            else { const int xx = lane - 9; xm = bx + (xx < 8 || ur ? xx : 7); ym = by - 1; av = up; }
            int v = 0;
            if (av) v = (xm >= 0 && xm < 16 && ym >= 0) ? q.rec8[ym * 16 + xm] : recY[(pix_y + ym) * W + pix_x + xm];
            q.raw[lane] = v;
            q.av[lane] = av;
        }
        for (int k = lane; k < 9 * (JMR_NCTX / 4) && !CAV; k += 64) {   // each rate lane's copy of the MB-start state
            const int m = k / (JMR_NCTX / 4), j = k - m * (JMR_NCTX / 4);
            reinterpret_cast<uint32_t *>(s.stc[m])[j] = reinterpret_cast<const uint32_t *>(s.st0)[j];
        }
        wave_lds_sync();
        if (lane < 25 && q.av[lane]) {
            const int c = q.raw[lane];
            const int lo = lane > 0 && q.av[lane - 1] ? q.raw[lane - 1] : c, hi = lane < 24 && q.av[lane + 1] ? q.raw[lane + 1] : c;
            q.f[lane] = (lo + 2 * c + hi + 2) >> 2;
        }
        // predIntra8x8PredMode (8.3.2.1): this MB's earlier blocks, else the neighbour's 4x4 mode
        const int ma = bx ? q.m8[b8 - 1] : s.bd.ipm[6 + (by >> 2)], mb = by ? q.m8[b8 - 2] : s.bd.ipm[1 + (bx >> 2)];
        const int mpm = (ma < 0 || mb < 0) ? 2 : min(ma, mb);
        wave_lds_sync();
        int st = 0, sl = 0;
        for (int i = 0; i < 8; i++) { st += up ? q.f[9 + i] : 0; sl += left ? q.f[i] : 0; }
        const int dcv = up && left ? (st + sl + 8) >> 4 : up ? (st + 4) >> 3 : left ? (sl + 4) >> 3 : (maxv + 1) >> 1;
        const int ov = s.org[(by + y) * 16 + bx + x];
#pragma unroll 1
        for (int m = 0; m < 9; m++) {                   // the nine modes' dct_luma8x8 (wave-uniform skips)
            const bool ok = m == 2 || ((m == 0 || m == 3 || m == 7) && up) || ((m == 1 || m == 8) && left) ||
                            ((m == 4 || m == 5 || m == 6) && up && left && ul);
            if (!ok) continue;
            const int p = i8_pred_px(q.f, dcv, m, x, y);
            const int c = wave_fwd8x8(ov - p, lane);
            int lev, dq, cost;
            const unsigned long long nz = wave_quant8(c, lane, qp, rnd, lev, dq, cost);
            const int rv = wave_inv8x8(dq, lane, p, maxv);
            q.lev8[m][lane] = (int16_t)lev;
            q.r8[m][lane] = (pel)rv;
            const int dist = wave_sum((ov - rv) * (ov - rv));
            if (lane == 0) { s.dist[m] = dist; s.nz[m] = nz != 0; }
        }
        wave_lds_sync();
        {                                               // lane m: the block's rate in mode m
            const int m = lane;
            const bool ok = m < 9 && (m == 2 || ((m == 0 || m == 3 || m == 7) && up) || ((m == 1 || m == 8) && left) ||
                                      ((m == 4 || m == 5 || m == 6) && up && left && ul));
            if (ok && CAV) s.bits[m] = jmv_i8(A, B, s.tcd, b8, m == mpm ? -1 : m < mpm ? m : m - 1, q.lev8[m], s.tcm[m]);
            else if (ok) {
                jmr_eng e = {s.stc[m], rg0, 0};
                jmr_i8(&e, m == mpm ? -1 : m < mpm ? m : m - 1, q.lev8[m]);
                s.bits[m] = e.bits;
            }
        }
        wave_lds_sync();
        double best = 1e30;                             // wave-uniform decision, strict '<'
        int bm = 2;
        for (int mm = 0; mm < 9; mm++) {
            const bool ok = mm == 2 || ((mm == 0 || mm == 3 || mm == 7) && up) || ((mm == 1 || mm == 8) && left) ||
                            ((mm == 4 || mm == 5 || mm == 6) && up && left && ul);
            if (!ok) continue;
            const double rd = rd_cost(s.dist[mm], s.bits[mm], d.lambda_rd);
            if (rd < best) { best = rd; bm = mm; }
        }
        q.rec8[(by + y) * 16 + bx + x] = q.r8[bm][lane];
        L.luma[il_blk(b8, lane)][lane >> 2] = q.lev8[bm][lane];
        if (lane == 0) {
            q.m8[b8] = bm;
            L.ipm[(b8 >> 1) * 8 + (b8 & 1) * 2] = (int8_t)(bm == mpm ? -1 : bm < mpm ? bm : bm - 1);
        }
        if (lane < 4) s.tcd[((b8 >> 1) * 2 + (lane >> 1)) * 4 + (b8 & 1) * 2 + (lane & 1)] = s.tcm[bm][lane];
        if (s.nz[bm]) { cbp |= 1 << b8; blkm |= 0x33 << ((b8 >> 1) * 8 + (b8 & 1) * 2); }
        wave_lds_sync();
    }
    int e2 = 0;
    for (int i = lane; i < 256; i += 64) {
        L.rec[i] = q.rec8[i];
        const int e = (int)s.org[i] - (int)q.rec8[i];
        e2 += e * e;
    }
    if (lane < 16) L.imode[lane] = (int8_t)q.m8[((lane >> 3) << 1) + ((lane & 3) >> 1)];
    if (lane < 32) L.mv[lane >> 1][lane & 1] = 0;
    const int dist = wave_sum(e2);
    if (lane == 0) { L.cbp = cbp; L.cbp_blk = blkm; L.dist = dist; L.i16mode = 0; }
}

template <class pel, bool T8, bool CAV>
__device__ __forceinline__ void rdo_intra_mb(const DevParams &d, RdoIntraS<pel, T8> &s, RdoScr<pel> *scr, int mbx, int mby, int lane) {
    const int a = mby * d.mbw + mbx, W = d.W, pix_x = 16 * mbx, pix_y = 16 * mby, qp = d.qp + d.qpbd, maxv = d.maxv;
    const MbAvail mav0 = mb_avail(d, mbx, mby), mav = intra_avail(d, mbx, mby);   // context neighbours / intra prediction
    const bool avL = mav.L, avT = mav.T, avTL = mav.TL, avTR = mav.TR;
    const bool prof = d.prof && lane == 0 && d.prof_mb == a;   // debug (JMH_PHASE_PROF): stamps 53..56
    PSTAMP(53);
    const pel *orgY = spl<pel>(d.orgY);
    for (int i = lane; i < 256; i += 64) s.org[i] = orgY[(pix_y + (i >> 4)) * W + pix_x + (i & 15)];
    for (int i = lane; i < 128; i += 64) load_orgc(d, s.nb, i, mbx, mby);
    for (int t = lane; t < 71; t += 64) load_intra_nb(d, s.nb, t, mbx, mby);
    if (lane >= 54 && lane < 64) load_border(d, s.bd, lane - 54, mbx, mby);
    const uint32_t rg0 = rdo_state_load(d, a, s.st0, lane, 64);
    jmr_lds_tables_load(lane, 64);
    {
        const int nw = (int)sizeof(jmr_mbinfo) / 4;
        if (lane < nw) {
            if (mav0.L) reinterpret_cast<uint32_t *>(&s.nbA)[lane] = reinterpret_cast<const uint32_t *>(d.rp->mbi + a - 1)[lane];
            if (mav0.T) reinterpret_cast<uint32_t *>(&s.nbB)[lane] = reinterpret_cast<const uint32_t *>(d.rp->mbi + a - d.mbw)[lane];
        }
    }
    wave_lds_sync();
    const jmr_mbinfo *A = mav0.L ? &s.nbA : nullptr, *B = mav0.T ? &s.nbB : nullptr;
    RdoLuma<pel> *L = scr->L;
    const int b4 = lane >> 4, l = lane & 15;
    // ---- Intra16x16: the find_sad_16x16 mode, dct_luma_16x16 a row of 4x4 blocks per pass (the DC
    //      Hadamard on lane 0, i16_dc)
    {
        int c16, m16;
        i16_pick(d, s.org, s.nb, lane, avL, avT, avTL, c16, m16);
        const pel *T = s.nb.rtop + 1, *Lf = s.nb.rleft;
        const I16Par par = i16_params(T, Lf, avT, avL, (maxv + 1) >> 1);
        const int rnd = q_round(q_sel16(d.qsel), 15 + qp / 6);
        int c[4], pr[4], o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int px4 = 4 * b4 + (l & 3), py4 = 4 * i + (l >> 2);
            pr[i] = i16_pred(par, T, Lf, m16, px4, py4, maxv);
            o[i] = s.org[py4 * 16 + px4];
            c[i] = lane_fwd4x4(o[i] - pr[i], l);
            if (l == 0) s.dc[4 * i + b4] = c[i];
        }
        wave_lds_sync();
        if (lane == 0) i16_dc(s.dc, s.dclev, s.dcdq, qp, rnd);
        wave_lds_sync();
        int e2 = 0, cbp = 0, blkm = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int blk = 4 * i + b4, px4 = 4 * b4 + (l & 3), py4 = 4 * i + (l >> 2);
            int lev, dq, cc;
            const unsigned nz = lane_quant(c[i], l, qp, rnd, true, lev, dq, cc);
            if (l == 0) dq = s.dcdq[blk];
            const int rv = lane_inv4x4(dq, l, pr[i], maxv);
            L[5].luma[blk][l] = (int16_t)lev;
            L[5].rec[py4 * 16 + px4] = (pel)rv;
            e2 += (o[i] - rv) * (o[i] - rv);
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (__builtin_amdgcn_readlane((int)nz, 16 * q)) { cbp = 15; blkm |= 1 << (4 * i + q); }
        }
        if (lane < 16) L[5].luma_dc[lane] = s.dclev[lane];
        if (lane < 32) L[5].mv[lane >> 1][lane & 1] = 0;
        const int dist = wave_sum(e2);
        if (lane == 0) { L[5].cbp = cbp; L[5].cbp_blk = blkm; L[5].dist = dist; L[5].i16mode = m16; }
    }
    PSTAMP(54);
    // ---- the four chroma intra modes (ChromaResidualCoding of IntraChromaPrediction8x8 [J])
#pragma unroll 1
    for (int m = 0; m < 4; m++) {
        const bool act = m == 0 || (m == 1 ? avL : m == 2 ? avT : avT && avL && avTL);
        if (!act) continue;                             // uniform
        const int dist = chroma_cand_w<pel>(d, s.nb.orgc[0], s.nb.orgc[1], 8, &s.nb, m, nullptr, false, &scr->C[5 + m], lane, mbx, mby, avT, avL);
        if (lane == 0) scr->C[5 + m].dist = dist;
    }
    // ---- Intra4x4: Mode_Decision_for_4x4IntraBlocks [J] by RDCost_for_4x4IntraBlocks, 16 blocks in
    //      coding order: 9 modes x 16 lanes code (three passes), lane m rates mode m, a wave-uniform
    //      decision
    PSTAMP(55);
    int i4cbp = 0, i4blk = 0;
    const int rnd = q_round(d.qsel, 15 + qp / 6);
    if (lane < 24) s.tcd[lane] = 0;
    int i4e[3];                                         // the lane's prediction formulas, once
#pragma unroll
    for (int pass = 0; pass < 3; pass++) i4e[pass] = 4 * pass + b4 < 9 ? c_i4tab[4 * pass + b4][l] : 0;
#pragma unroll 1
    for (int i = 0; i < 16; i++) {
        const int b8 = i >> 2, bb = i & 3;
        const int bx = 8 * (b8 & 1) + 4 * (bb & 1), by = 8 * (b8 >> 1) + 4 * (bb >> 1), bx4 = bx >> 2, by4 = by >> 2, blk = 4 * by4 + bx4;
        const bool up = by > 0 || avT, left = bx > 0 || avL;
        const bool ul = (bx > 0 && by > 0) || (bx == 0 && by > 0 && avL) || (bx > 0 && by == 0 && avT) || (bx == 0 && by == 0 && avTL);
        bool ur = by == 0 ? (bx + 4 <= 15 ? avT : avTR) : (bx + 4 <= 15);
        if ((bx == 4 || bx == 12) && (by == 4 || by == 12)) ur = false;
        if (lane < 13) {
            int v;
            if (lane == 0) v = ul ? i4_lpix(s, bx - 1, by - 1) : 0;
            else if (lane <= 4) v = up ? i4_lpix(s, bx + lane - 1, by - 1) : 0;
            else if (lane <= 8) v = up ? i4_lpix(s, ur ? bx + lane - 1 : bx + 3, by - 1) : 0;
            else v = left ? i4_lpix(s, bx - 1, by + lane - 9) : 0;
            s.P[lane] = v;
        }
        const int upM = by > 0 ? s.ipred_cur[blk - 4] : s.bd.ipm[1 + bx4];
        const int leftM = bx > 0 ? s.ipred_cur[blk - 1] : s.bd.ipm[6 + by4];
        const int mpm = (upM < 0 || leftM < 0) ? 2 : min(upM, leftM);
        for (int k = lane; k < 9 * (JMR_NCTX / 4) && !CAV; k += 64) {   // each rate lane's copy of the MB-start state
            const int m = k / (JMR_NCTX / 4), j = k - m * (JMR_NCTX / 4);
            reinterpret_cast<uint32_t *>(s.stc[m])[j] = reinterpret_cast<const uint32_t *>(s.st0)[j];
        }
        wave_lds_sync();
        const int org = s.org[(by + (l >> 2)) * 16 + bx + (l & 3)];
        const int st = s.P[1] + s.P[2] + s.P[3] + s.P[4], sl = s.P[9] + s.P[10] + s.P[11] + s.P[12];
        const int dcp = (up && left) ? (st + sl + 4) >> 3 : left ? (sl + 2) >> 2 : up ? (st + 2) >> 2 : (maxv + 1) >> 1;
#pragma unroll
        for (int pass = 0; pass < 3; pass++) {          // the nine modes' dct_luma
            const int m = 4 * pass + b4;
            if (pass == 2 && b4 > 0) break;             // wave-uniform per 16-lane row; DPP stays inside rows
            const int e = i4e[pass], ty = e & 3;
            const int pa = s.P[(e >> 2) & 15], pb = s.P[(e >> 6) & 15], pc = s.P[(e >> 10) & 15];
            const int p = ty == 1 ? (pa + pb + 1) >> 1 : ty == 2 ? (pa + 2 * pb + pc + 2) >> 2 : dcp;
            const int c = lane_fwd4x4(org - p, l);
            int lev, dq, cc;
            const unsigned nz = lane_quant(c, l, qp, rnd, false, lev, dq, cc);
            const int rv = lane_inv4x4(dq, l, p, maxv);
            s.lev[m][l] = (int16_t)lev;
            s.r4[m][l] = (pel)rv;
            const int dist = row16_sum((org - rv) * (org - rv));
            if (l == 0) { s.dist[m] = dist; s.nz[m] = nz != 0; }
        }
        wave_lds_sync();
        {                                               // lane m: the block's rate in mode m
            const int m = lane;
            const bool avm = m < 9 && (m == 2 || ((m == 0 || m == 3 || m == 7) && up) || ((m == 1 || m == 8) && left) || (up && left && ul));
            if (avm && CAV) {
                int tc;
                s.bits[m] = jmv_i4(A, B, s.tcd, bx4, by4, m == mpm ? -1 : m < mpm ? m : m - 1, s.lev[m], &tc);
                s.tcm[m][0] = (uint8_t)tc;
            } else if (avm) {
                jmr_eng e = {s.stc[m], rg0, 0};
                jmr_i4(&e, A, B, bx4, by4, m == mpm ? -1 : m < mpm ? m : m - 1, s.lev[m]);
                s.bits[m] = e.bits;
            }
        }
        wave_lds_sync();
        double best = 1e30;                             // wave-uniform decision, strict '<'
        int bm = 2;
        for (int mm = 0; mm < 9; mm++) {
            const bool av = mm == 2 || ((mm == 0 || mm == 3 || mm == 7) && up) || ((mm == 1 || mm == 8) && left) || (up && left && ul);
            if (!av) continue;
            const double rd = rd_cost(s.dist[mm], s.bits[mm], d.lambda_rd);
            if (rd < best) { best = rd; bm = mm; }
        }
        if (lane == 0) {
            s.tcd[blk] = s.tcm[bm][0];
            s.ipred_cur[blk] = (int8_t)bm;
            L[6].imode[blk] = (int8_t)bm;
            L[6].ipm[blk] = (int8_t)(bm == mpm ? -1 : bm < mpm ? bm : bm - 1);
        }
        if (s.nz[bm]) { i4cbp |= 1 << b8; i4blk |= 1 << blk; }
        if (lane < 16) {
            s.rec[(by + (lane >> 2)) * 16 + bx + (lane & 3)] = s.r4[bm][lane];
            L[6].luma[blk][lane] = s.lev[bm][lane];
        }
        wave_lds_sync();
    }
    int e2 = 0;
    for (int i = lane; i < 256; i += 64) {
        L[6].rec[i] = s.rec[i];
        const int e = (int)s.org[i] - (int)s.rec[i];
        e2 += e * e;
    }
    const int dist = wave_sum(e2);
    if (lane == 0) { L[6].cbp = i4cbp; L[6].cbp_blk = i4blk; L[6].dist = dist; L[6].i16mode = 0; }
    if (lane < 32) L[6].mv[lane >> 1][lane & 1] = 0;
    if constexpr (T8) {
        if (lane < 24) s.tcd[lane] = 0;
        wave_lds_sync();
        rdo_intra8<pel, CAV>(d, s, L[7], A, B, rg0, mav, mbx, mby, lane);
    }
    PSTAMP(56);
    // ---- RDCost_for_macroblocks' rate of the eight intra candidates (I16MB / I4MB x the chroma
    //      modes; Transform8x8Mode: and I8MB), here beside k_rdo_inter rather than on k_rdo_final's
    //      critical path: lane k < 8 (12) codes candidate k on its own copy of the slice state (the
    //      Intra4x4 copies, free now), reading the candidates this wave wrote to the tick scratch
    constexpr int NI = T8 ? 12 : 8;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int k = lane; k < NI * (JMR_NCTX / 4) && !CAV; k += 64) {
        const int m = k / (JMR_NCTX / 4), j = k - m * (JMR_NCTX / 4);
        reinterpret_cast<uint32_t *>(s.stc[m])[j] = reinterpret_cast<const uint32_t *>(s.st0)[j];
    }
    wave_lds_sync();
    const int cm = lane & 3;
    const bool cok = cm == 0 || (cm == 1 ? avL : cm == 2 ? avT : avT && avL && avTL);
    if (lane < NI && cok) {
        const RdoLuma<pel> &Lc = L[5 + (lane >> 2)];
        const RdoChroma<pel> &C = scr->C[5 + cm];
        RdoRate &R = scr->R[lane];
        jmr_cand r;
        r.mb_type = lane < 4 ? JMH_I16MB : lane < 8 ? JMH_I4MB : JMH_I8MB;
        r.cbp = Lc.cbp | C.cbpc << 4;
        r.i16mode = Lc.i16mode;
        r.cmode = cm;
        r.t8 = lane >= 8;
        for (int q = 0; q < 4; q++) r.b8mode[q] = 0;
        r.ipm = Lc.ipm;
        r.mvd = Lc.mvd;
        r.luma = Lc.luma;
        r.luma_dc = Lc.luma_dc;
        r.cdc = C.dc;
        r.cac = C.ac;
        r.mvw = R.mvw;
        if (CAV) {                                  // rg0: the mb_skip_run before this macroblock
            R.bits = jmv_mb(A, B, &r, d.slice_type == JMH_P_SLICE, T8, (int)rg0, reinterpret_cast<uint8_t *>(R.mvw), &R.out);
            R.range = 0;
        } else {
            jmr_eng en = {s.stc[lane], rg0, 0};
            jmr_mb(&en, A, B, &r, d.slice_type == JMH_P_SLICE, T8, &R.out);
            R.bits = en.bits;
            R.range = en.range;
        }
    }
    wave_lds_sync();
    for (int k = lane; k < NI * (JMR_NCTX / 4) && !CAV; k += 64) {
        const int m = k / (JMR_NCTX / 4), j = k - m * (JMR_NCTX / 4);
        reinterpret_cast<uint32_t *>(scr->R[m].ctx)[j] = reinterpret_cast<const uint32_t *>(s.stc[m])[j];
    }
    PSTAMP(61);
}

#ifndef JMH_RDO_INTER_WPE
#define JMH_RDO_INTER_WPE 1                   // waves per SIMD the register budget must allow (2: five per CU
#endif                                        //   at 16 bits, 32 B of scratch, 10 % slower: profiles/r7x_fallback_ab.txt)
template <class pel, bool T8, bool FFS>
__global__ __launch_bounds__(NTE, JMH_RDO_INTER_WPE) void k_rdo_inter(const TickArgs t) {
    __shared__ RdoInterS<pel> s;
    const int nP = t.pre[t.nP], m = xcd_block(blockIdx.x, nP);
    if (m >= nP) return;                                // padding block (whole workgroup)
    // the inter role is the tick's long pole; the intra role's waves sharing its SIMDs (side
    // stream) take the issue slots it leaves
    __builtin_amdgcn_s_setprio(3);
    const unsigned long long bt0 = t.bprof ? wall_clock64() : 0;   // debug (JMH_BLOCK_PROF): role 4
    const int e = tick_entry(t, m);
    const DevParams d = tick_params(t, e);
    int mbx, mby;
    tick_mb(t, d, e, m, mbx, mby);
    // SearchMode 0: the MB's SAD table in the tick slot's (ffs_slot_bytes; null: every search scans)
    uint8_t *ftab = t.ffs ? reinterpret_cast<uint8_t *>(t.ffs) + (size_t)m * t.ffs_slot : nullptr;
    rdo_inter_mb<pel, T8, FFS>(d, s, reinterpret_cast<RdoScr<pel> *>(t.rscr) + m, ftab, mbx, mby, threadIdx.x);
    if (t.bprof && threadIdx.x == 0) {
        t.bprof[3 * blockIdx.x] = bt0;
        t.bprof[3 * blockIdx.x + 1] = wall_clock64();
        t.bprof[3 * blockIdx.x + 2] = 4;
    }
}
// CAV: SymbolMode 0 (the CAVLC rates; the CABAC build keeps its registers)
template <class pel, bool T8, bool CAV>
__global__ __launch_bounds__(NTE) void k_rdo_intra(const TickArgs t) {
    __shared__ RdoIntraS<pel, T8> s;
    const int tot = t.pre[t.npic], m = xcd_block(blockIdx.x, tot);
    if (m >= tot) return;
    const unsigned long long bt0 = t.bprof ? wall_clock64() : 0;   // debug (JMH_BLOCK_PROF): role 1
    const int e = tick_entry(t, m);
    const DevParams d = tick_params(t, e);
    int mbx, mby;
    tick_mb(t, d, e, m, mbx, mby);
    rdo_intra_mb<pel, T8, CAV>(d, s, reinterpret_cast<RdoScr<pel> *>(t.rscr) + m, mbx, mby, threadIdx.x);
    if (t.bprof && threadIdx.x == 0) {
        unsigned long long *bp = t.bprof + 3 * xcd_grid(t.pre[t.nP]);
        bp[3 * blockIdx.x] = bt0;
        bp[3 * blockIdx.x + 1] = wall_clock64();
        bp[3 * blockIdx.x + 2] = 1;
    }
}

// ======================================================================================
//  k_rdo_final: RDCost_for_macroblocks over the candidates, the decision, its outputs
// ======================================================================================
struct RdoFinL {                  // the syntax of a luma candidate the rate reads (RdoLuma's first 672 B + ipm)
    int16_t luma[16][16];
    int16_t luma_dc[16];
    int16_t mv[16][2];
    int16_t mvd[16][2];
    int8_t ipm[16];
};
struct RdoFinC {                  // of a chroma candidate (RdoChroma's first 272 B)
    int16_t dc[2][4];
    int16_t ac[2][4][16];
};
// the inter candidates' LDS syntax slot: 0..4 and (Transform8x8Mode) 8..11 -> 5..8
__device__ __forceinline__ int rd_fslot(int i) { return i < 5 ? i : i - 3; }
template <class pel>
struct RdoFinS {
    RdoFinL fl[9];                // the inter candidates' syntax in LDS: the serial CABAC loops read it bin by bin
    RdoFinC fc[5];
    int16_t mvw[RD_NCAND][16][2];   // jmr_mb's work buffers
    alignas(4) uint8_t st0[JMR_NCTX];
    alignas(4) uint8_t stc[RD_NCAND][JMR_NCTX];
    jmr_mbinfo nbA, nbB, out[RD_NCAND];
    int hasA, hasB;
    uint32_t rg0, rgo[RD_NCAND];
    double rd[RD_NCAND];
    int bits[RD_NCAND], ci[RD_NCAND], ccm[RD_NCAND];
    int8_t kof[4][4];             // the candidate on lane j < 4 of wave w (-1: none)
    int ncand, win;
    alignas(4) pel rec[256];
    pel cfin[2][64];
    int16_t fmv[16][2];
    DbkS<pel> db;
};

// T8: Transform8x8Mode (the 8x8-transform and I8MB candidates; jmr_mb's 8x8 residual path); CAV:
// SymbolMode 0 (jmv_mb rates, the slice's mb_skip_run)
#ifndef JMH_RDO_FINAL_WPE
#define JMH_RDO_FINAL_WPE 5                   // Transform8x8Mode: waves per SIMD the register budget must allow
#endif                                        //   (the 8x8 CABAC residual path would take 146 VGPRs: three)
template <class pel, bool T8, bool CAV>
__global__ __launch_bounds__(NT, T8 ? JMH_RDO_FINAL_WPE : 1) void k_rdo_final(const TickArgs t) {
    __shared__ RdoFinS<pel> s;
    const int tid = threadIdx.x, tot = t.pre[t.npic];
    const int m = xcd_block(blockIdx.x, tot);
    if (m >= tot) return;
    const unsigned long long bt0 = t.bprof_fin ? wall_clock64() : 0;   // debug (JMH_BLOCK_PROF): role 3
    const int e = tick_entry(t, m);
    const DevParams d = tick_params(t, e);
    int mbx, mby;
    tick_mb(t, d, e, m, mbx, mby);
    const RdoScr<pel> *scr = reinterpret_cast<const RdoScr<pel> *>(t.rscr) + m;
    const int a = mby * d.mbw + mbx, W = d.W, Wc = d.Wc, W4 = d.W >> 2, pix_x = 16 * mbx, pix_y = 16 * mby;
    const bool prof = d.prof && tid == 0 && d.prof_mb == a;   // debug (JMH_PHASE_PROF): stamps 57..60
    PSTAMP(57);
    const bool slice_p = d.slice_type == JMH_P_SLICE;
    const MbAvail mav = intra_avail(d, mbx, mby);       // (the chroma modes' availability)
    if (tid < 64) {
        const uint32_t rg = rdo_state_load(d, a, s.st0, tid, 64);
        if (tid == 0) s.rg0 = rg;
    } else if (tid < 128) rdo_nb_load(d, mbx, mby, s.nbA, s.nbB, s.hasA, s.hasB, tid - 64);
    else if (tid >= 160) jmr_lds_tables_load(tid - 160, 96);
    else if (tid == 128) {                              // the candidates in JM's order (item 63 with Transform8x8Mode)
        const bool p8 = inter_on(d.isr, 4) || inter_on(d.isr, 5) || inter_on(d.isr, 6) || inter_on(d.isr, 7);
        const bool p8t8 = T8 && p8 && scr->L[4].b8mode[0] == 4 && scr->L[4].b8mode[1] == 4 && scr->L[4].b8mode[2] == 4 &&
                          scr->L[4].b8mode[3] == 4;
        const bool cav[4] = {true, mav.L, mav.T, mav.T && mav.L && mav.TL};
        static constexpr int8_t order[RD_NL] = {0, 1, 8, 2, 9, 3, 10, 4, 11, 5, 6, 7};
        int n = 0;
        for (int cm = 0; cm < 4; cm++) {
            if (!cav[cm]) continue;
            for (int oi = 0; oi < RD_NL; oi++) {
                const int i = order[oi], b = rd_cbase(i);
                const bool intra = i >= 5 && i <= 7;
                bool valid = intra ? (i < 7 || T8) : slice_p && (b == 0 || (b == 4 ? p8 : inter_on(d.isr, b)));
                if (i >= 8) valid = valid && T8 && (i != 11 || p8t8);
                if (!valid || (cm != 0 && !intra)) continue;
                s.ci[n] = i; s.ccm[n] = cm; n++;
            }
        }
        s.ncand = n;
        // the inter candidates' rates, one per wave (lanes of a wave in different syntax would cost
        // the sum of their paths): wave 0 16x16, 1 16x8, 2 8x16 and P_Skip, 3 P8x8, each with both
        // transform sizes; the intra candidates' rates come from k_rdo_intra (RdoScr.R)
        int fill[4] = {0, 0, 0, 0};
        for (int w = 0; w < 16; w++) s.kof[w >> 2][w & 3] = -1;
        for (int k = 0; k < n; k++) {
            const int i = s.ci[k], b = rd_cbase(i);
            if (i >= 5 && i <= 7) continue;
            const int w = b == 1 ? 0 : b == 2 ? 1 : b == 4 ? 3 : 2;
            s.kof[w][fill[w]++] = (int8_t)k;
        }
    }
    __syncthreads();
    const jmr_mbinfo *A = s.hasA ? &s.nbA : nullptr, *B = s.hasB ? &s.nbB : nullptr;
    // ---- one lane per candidate: its rate on its own copy of the coding state (lanes 0..3 of the
    //      four waves, grouped by macroblock type: kof)
    for (int i = tid; i < s.ncand * (JMR_NCTX / 4) && !CAV; i += NT) {   // the inter candidates' state copies
        const int k = i / (JMR_NCTX / 4), j = i - k * (JMR_NCTX / 4), ci = s.ci[k];
        if (ci < 5 || ci >= 8) reinterpret_cast<uint32_t *>(s.stc[k])[j] = reinterpret_cast<const uint32_t *>(s.st0)[j];
    }
    {
        constexpr int nl = 672 / 4, nc = (int)sizeof(RdoFinC) / 4;
        static_assert(offsetof(RdoLuma<pel>, ipm) > 672 && offsetof(RdoFinL, ipm) == 672, "RdoFinL layout");
        const int nfl = T8 ? 9 : 5;
        for (int i = tid; i < nfl * (nl + 4); i += NT) {
            const int f = i / (nl + 4), j = i - f * (nl + 4), k = f < 5 ? f : f + 3;
            const uint32_t *src = reinterpret_cast<const uint32_t *>(&scr->L[k]);
            reinterpret_cast<uint32_t *>(&s.fl[f])[j] = j < nl ? src[j] : reinterpret_cast<const uint32_t *>(scr->L[k].ipm)[j - nl];
        }
        for (int i = tid; i < 5 * nc; i += NT) {
            const int k = i / nc, j = i - k * nc;
            reinterpret_cast<uint32_t *>(&s.fc[k])[j] = reinterpret_cast<const uint32_t *>(&scr->C[k])[j];
        }
        // the intra candidates: their rates as k_rdo_intra coded them
        const int nw = (int)sizeof(jmr_mbinfo) / 4;
        for (int i = tid; i < s.ncand * (nw + 2); i += NT) {
            const int k = i / (nw + 2), j = i - k * (nw + 2), ci = s.ci[k];
            if (ci < 5 || ci > 7) continue;
            const RdoRate &R = scr->R[4 * (ci - 5) + s.ccm[k]];
            if (j < nw) reinterpret_cast<uint32_t *>(&s.out[k])[j] = reinterpret_cast<const uint32_t *>(&R.out)[j];
            else if (j == nw) s.rgo[k] = R.range;
            else {
                s.bits[k] = R.bits;
                s.rd[k] = rd_cost(scr->L[ci].dist + scr->C[5 + s.ccm[k]].dist, R.bits, d.lambda_rd);
            }
        }
    }
    __syncthreads();
    PSTAMP(58);
    const int kc = (tid & 63) < 4 ? s.kof[tid >> 6][tid & 3] : -1;
    if (kc >= 0) {
        const int i = s.ci[kc], b = rd_cbase(i);
        const RdoLuma<pel> &L = scr->L[i];
        const RdoChroma<pel> &C = scr->C[b];
        jmr_eng en = {s.stc[kc], s.rg0, 0};
        if (i == 0) {
            if (CAV) {                          // P_Skip: its run is written with the next coded MB (rate 0), or
                s.out[kc] = jmr_mbinfo{};       //   by this MB when it is the picture's last (item 64(a))
                en.bits = jmv_skip((int)s.rg0, a == d.mbw * d.mbh - 1);
            }
            else jmr_skip(&en, A, B, &s.out[kc]);
        } else {
            jmr_cand r;
            r.mb_type = b == 4 ? JMH_P8x8 : b;
            r.cbp = L.cbp | C.cbpc << 4;
            r.i16mode = L.i16mode;
            r.cmode = 0;
            r.t8 = T8 && i >= 8;
            for (int q = 0; q < 4; q++) r.b8mode[q] = L.b8mode[q];
            const RdoFinL &FL = s.fl[rd_fslot(i)];
            const RdoFinC &FC = s.fc[b];
            r.ipm = FL.ipm;
            r.mvd = FL.mvd;
            r.luma = FL.luma;
            r.luma_dc = FL.luma_dc;
            r.cdc = FC.dc;
            r.cac = FC.ac;
            r.mvw = s.mvw[kc];
            if (CAV) en.bits = jmv_mb(A, B, &r, slice_p, T8, (int)s.rg0, reinterpret_cast<uint8_t *>(s.mvw[kc]), &s.out[kc]);
            else jmr_mb(&en, A, B, &r, slice_p, T8, &s.out[kc]);
        }
        s.bits[kc] = en.bits;
        s.rgo[kc] = en.range;
        s.rd[kc] = rd_cost(L.dist + C.dist, en.bits, d.lambda_rd);
    }
    __syncthreads();
    PSTAMP(59);
    if (tid == 0) {                                     // strict '<' in JM's order
        double best = 1e30;
        int w = 0;
        for (int k = 0; k < s.ncand; k++)
            if (s.rd[k] < best) { best = s.rd[k]; w = k; }
        s.win = w;
    }
    __syncthreads();
    // ---- the chosen macroblock: results, reconstruction, picture arrays, coding state
    const int w = s.win, bi = s.ci[w], bcm = s.ccm[w], bb = rd_cbase(bi);
    const RdoLuma<pel> &L = scr->L[bi];
    const bool is_intra = bi >= 5 && bi <= 7;
    const RdoChroma<pel> &C = scr->C[is_intra ? 5 + bcm : bb];
    const int mb_type = bi == 0 ? JMH_PSKIP : bb == 4 ? JMH_P8x8 : bi == 5 ? JMH_I16MB : bi == 6 ? JMH_I4MB : bi == 7 ? JMH_I8MB : bb;
    const int cbp = L.cbp | C.cbpc << 4, cbp_blk = L.cbp_blk;
    const bool tr8 = T8 && rd_t8(bi) && (mb_type == JMH_I8MB || (cbp & 15));   // transform_size_8x8_flag
    jmh_mb_result *res = d.res + a;
    if (tid == 0) {
        res->mb_type = (int16_t)mb_type;
        res->cbp = (int16_t)cbp;
        res->cbp_blk = cbp_blk;
        for (int q = 0; q < 4; q++) {
            res->b8mode[q] = (int8_t)(mb_type == JMH_PSKIP ? 0 : mb_type == JMH_P8x8 ? L.b8mode[q] : mb_type == JMH_I4MB ? JMH_IBLOCK
                                                       : mb_type == JMH_I16MB ? 0 : mb_type);
            res->ref_idx[q] = (int8_t)(is_intra ? -1 : 0);
        }
        res->i16mode = (int8_t)(mb_type == JMH_I16MB ? L.i16mode : 0);
        res->c_ipred_mode = (int8_t)(is_intra ? bcm : 0);
        res->transform_8x8 = (int8_t)tr8; res->pad0 = 0;
        res->min_cost = s.bits[w];                      // the chosen candidate's rate (bits)
        res->reserved = 0;
    }
    const int blk = tid >> 4, l = tid & 15;
    res->luma[blk][l] = L.luma[blk][l];
    if (tid < 16) {
        const int k = tid;
        const int ip = mb_type == JMH_I4MB || mb_type == JMH_I8MB ? L.imode[k] : 2;
        const int mx = is_intra ? 0 : L.mv[k][0], my = is_intra ? 0 : L.mv[k][1];
        res->ipred[k] = (int8_t)ip;
        res->mv[k][0] = (int16_t)mx; res->mv[k][1] = (int16_t)my;
        res->luma_dc[k] = mb_type == JMH_I16MB ? L.luma_dc[k] : 0;
        s.fmv[k][0] = (int16_t)mx; s.fmv[k][1] = (int16_t)my;
        const int pa = ((pix_y >> 2) + (k >> 2)) * W4 + (pix_x >> 2) + (k & 3);
        d.mv[2 * pa] = (int16_t)mx; d.mv[2 * pa + 1] = (int16_t)my;
        d.refidx[pa] = (int8_t)(is_intra ? -1 : 0);
        d.ipred[pa] = (int8_t)ip;
    }
    if (tid < 8) res->chroma_dc[tid >> 2][tid & 3] = C.dc[tid >> 2][tid & 3];
    pel *recY = spl<pel>(d.recY), *recU = spl<pel>(d.recU), *recV = spl<pel>(d.recV);
    const pel rv = L.rec[tid];
    s.rec[tid] = rv;
    recY[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)] = rv;
    if (tid < 128) {
        const int uv = tid >> 6, k = tid & 63;
        res->chroma_ac[uv][k >> 4][k & 15] = C.ac[uv][k >> 4][k & 15];
        const pel cv = C.rec[uv][k];
        s.cfin[uv][k] = cv;
        (uv ? recV : recU)[((pix_y >> 1) + (k >> 3)) * Wc + (pix_x >> 1) + (k & 7)] = cv;
    }
    // write_one_macroblock: the slice's coding state advances by the chosen candidate, then its
    // end_of_slice_flag = 0 unless the slice ends here
    {
        const int slice = a / d.slice_mbs;
        uint32_t *dst = reinterpret_cast<uint32_t *>(d.rp->cab + (size_t)slice * JMR_NCTX);
        const uint8_t *win_ctx = is_intra ? scr->R[4 * (bi - 5) + bcm].ctx : s.stc[w];
        if (tid < JMR_NCTX / 4 && !CAV) dst[tid] = reinterpret_cast<const uint32_t *>(win_ctx)[tid];
        const int nw = (int)sizeof(jmr_mbinfo) / 4;
        if (tid >= 128 && tid < 128 + nw)
            reinterpret_cast<uint32_t *>(d.rp->mbi + a)[tid - 128] = reinterpret_cast<const uint32_t *>(&s.out[w])[tid - 128];
        if (tid == 192 && CAV) d.rp->range[slice] = bi == 0 ? s.rg0 + 1 : 0;   // mb_skip_run
        else if (tid == 192) {
            jmr_eng en = {nullptr, s.rgo[w], 0};
            if ((a + 1) % d.slice_mbs != 0 && a + 1 < d.mbw * d.mbh) jmr_end_of_mb(&en);
            d.rp->range[slice] = en.range;
        }
    }
    // ---- DeblockMb [J] (jmh_deblock.h)
    if (d.dbkY) {
        const int qpi = iclip(-d.qpbd, 51, d.qp + d.cqp_off), qpcy = qpi < 0 ? qpi : c_qpc[qpi];
        deblock_mb(d, s.db, s.rec, s.cfin, s.fmv, is_intra, cbp_blk, tr8, d.qp, qpcy, mbx, mby, tid);
    }
    PSTAMP(60);
    if (t.bprof_fin && tid == 0) {
        t.bprof_fin[3 * blockIdx.x] = bt0;
        t.bprof_fin[3 * blockIdx.x + 1] = wall_clock64();
        t.bprof_fin[3 * blockIdx.x + 2] = 3;
    }
}

// the instantiation of k_rdo_intra / k_rdo_final for the sample type, Transform8x8Mode and SymbolMode
typedef void (*RdoKern)(const TickArgs);
template <bool W, bool T8>
static RdoKern rdo_pick(bool fin, bool cav) {
    typedef typename std::conditional<W, uint16_t, uint8_t>::type pel;
    if (fin) return cav ? k_rdo_final<pel, T8, true> : k_rdo_final<pel, T8, false>;
    return cav ? k_rdo_intra<pel, T8, true> : k_rdo_intra<pel, T8, false>;
}
static RdoKern rdo_pick(bool wide, bool t8, bool fin, bool cav) {
    return wide ? (t8 ? rdo_pick<true, true>(fin, cav) : rdo_pick<true, false>(fin, cav))
                : (t8 ? rdo_pick<false, true>(fin, cav) : rdo_pick<false, false>(fin, cav));
}

// one tick: k_rdo_inter and k_rdo_intra (on the side stream when given: fork / join events), then
// k_rdo_final
hipError_t jmh_launch_rdo(const TickArgs &t, hipStream_t st, hipStream_t side, hipEvent_t fork, hipEvent_t join) {
    const int tot = t.pre[t.npic];
    if (!tot) return hipSuccess;
    const int nP = t.pre[t.nP];
    hipError_t err;
    hipStream_t ist = side ? side : st;
    if (side && nP) {
        if ((err = hipEventRecord(fork, st)) != hipSuccess || (err = hipStreamWaitEvent(side, fork, 0)) != hipSuccess) return err;
    } else ist = st;
    // Transform8x8Mode / SymbolMode 0: the instantiations with the 8x8-transform candidates / the
    // CAVLC rates (the others keep their registers and LDS)
    typedef void (*Kern)(const TickArgs);
    const Kern kin = t.ffs ? (t.bd > 8 ? (t.t8 ? k_rdo_inter<uint16_t, true, true> : k_rdo_inter<uint16_t, false, true>)
                                       : (t.t8 ? k_rdo_inter<uint8_t, true, true> : k_rdo_inter<uint8_t, false, true>))
                           : (t.bd > 8 ? (t.t8 ? k_rdo_inter<uint16_t, true, false> : k_rdo_inter<uint16_t, false, false>)
                                       : (t.t8 ? k_rdo_inter<uint8_t, true, false> : k_rdo_inter<uint8_t, false, false>));
    const bool cav = t.rdo == 2;
    const Kern kia = rdo_pick(t.bd > 8, t.t8 != 0, false, cav);
    if (nP) hipLaunchKernelGGL(kin, dim3(xcd_grid(nP)), dim3(NTE), 0, st, t);
    hipLaunchKernelGGL(kia, dim3(xcd_grid(tot)), dim3(NTE), 0, ist, t);
    if ((err = hipGetLastError()) != hipSuccess) return err;
    if (ist != st) {
        if ((err = hipEventRecord(join, ist)) != hipSuccess || (err = hipStreamWaitEvent(st, join, 0)) != hipSuccess) return err;
    }
    const Kern kfi = rdo_pick(t.bd > 8, t.t8 != 0, true, cav);
    hipLaunchKernelGGL(kfi, dim3(xcd_grid(tot)), dim3(NT), 0, st, t);
    return hipGetLastError();
}
