// jmh_rdo.hip — encode_one_macroblock with RDOptimization = 1 [J] on the device (row f4, config 5):
// the rate-distortion loop of rdopt.c (RDCost_for_macroblocks, RDCost_for_8x8blocks,
// RDCost_for_4x4IntraBlocks) with J = SSD + lambda * R and R the CABAC rate of the slice's coding
// state (jmh_cabac_rate.h, shared with the CPU oracle oracle/rdo.c).  DESIGN.md §9 has the
// schedule; one tick of the RD stage schedule runs
//   k_rdo_analyse  role "inter" (P MBs): the EPZS searches (wave 0), P8x8 block by block with the
//                  four sub-modes coded and rated on the four waves, the residual coding of the
//                  skip / 16x16 / 16x8 / 8x16 / P8x8 candidates and their chroma;
//                  role "intra" (all MBs): Intra16x16, the four chroma intra modes, Intra4x4 by
//                  per-block RD (9 modes x 16 lanes code, 9 lanes rate);
//   k_rdo_final    all MBs: one lane per macroblock candidate rates it on its own LDS copy of the
//                  contexts, the strict-'<' minimum of D + lambda R in JM's order wins; results,
//                  reconstruction, the slice's next coding state, the fused DeblockMb.
// Candidates travel between the two launches through the tick's scratch (RdoScr, HBM).
// docs/JM_SEMANTICS.md items 53-60 pin every RD choice.
#include "jmh_epzs.h"
#include "jmh_intra.h"
#include "jmh_deblock.h"
#include "jmh_cabac_rate.h"

#define RD_NL 7       // luma candidates: 0 P_Skip, 1 16x16, 2 16x8, 3 8x16, 4 P8x8, 5 I16MB, 6 I4MB
#define RD_NCAND 13   // macroblock-loop candidates: 5 inter + (I16, I4) x 4 chroma modes

// J = D + lambda * R in double, no contraction (the oracle's gcc x86-64 build has none either)
__device__ __forceinline__ double rd_cost(int dist, int bits, double lambda) {
#pragma clang fp contract(off)
    return (double)dist + lambda * (double)bits;
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
template <class pel>
struct RdoScr {
    RdoLuma<pel> L[RD_NL];
    RdoChroma<pel> C[9];          // [0..4]: chroma of L[0..4]; [5 + m]: intra chroma mode m
};
size_t jmh_rdo_scratch_bytes() { return sizeof(RdoScr<uint16_t>); }

// chroma-coding scratch of one candidate on 128 threads
struct ChromaBuf {
    int cdcin[2][4], cbcost[2][4], cbnz[2][4], cdcq[2][4], creset[2], cdcnz[2], red[2];
    int16_t cdc[2][4];
};

// the coding state of the slice at the start of macroblock a into st (LDS, 4-aligned) by threads
// [0, n): initialised (9.3.1.1) at the slice's first macroblock; returns codIRange
__device__ __forceinline__ uint32_t rdo_state_load(const DevParams &d, int a, uint8_t *st, int t, int n) {
    const int slice = a / d.slice_mbs;
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
__device__ __forceinline__ void copy_ctx(uint8_t *dst, const uint8_t *src) {   // one lane, 72 dwords
    for (int i = 0; i < JMR_NCTX / 4; i++) reinterpret_cast<uint32_t *>(dst)[i] = reinterpret_cast<const uint32_t *>(src)[i];
}
// sum over the 256 threads (every thread gets it); red: 4 ints of LDS
__device__ __forceinline__ int block_sum(int v, int *red, int tid) {
    v = wave_sum(v);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// ChromaResidualCoding [J] of one candidate on 128 threads (t = 0..127): prediction = intra mode cm
// (nb) or the MC of fmv; skipped (P_Skip): no residual.  act = false: the threads only take part
// in the barriers.  Writes out (global) except its distortion, returned on every thread.
template <class pel>
__device__ __forceinline__ int chroma_cand(const DevParams &d, const pel (*orgc)[64], const IntraNb<pel> *nb, int cm, const int16_t (*fmv)[2],
                                           bool skipped, bool act, ChromaBuf &cb, RdoChroma<pel> *out, int t, int mbx, int mby,
                                           bool avT, bool avL) {
    const int maxv = d.maxv, Wc = d.Wc, pix_x = 16 * mbx, pix_y = 16 * mby;
    const int qpi = iclip(-d.qpbd, 51, d.qp + d.cqp_off), qpcy = qpi < 0 ? qpi : c_qpc[qpi], qpc = qpcy + d.qpbd;
    const int cq_bits = 15 + qpc / 6, cqp_const = q_round(d.qsel, cq_bits);
    const int uv = t >> 6, cb4 = (t >> 4) & 3, l = t & 15;
    const int cxo = (cb4 & 1) * 4 + (l & 3), cyo = (cb4 >> 1) * 4 + (l >> 2);
    int pv = 0, lev = 0, cdq = 0;
    if (act) {
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
        if (!skipped) {
            const int c = lane_fwd4x4(orgc[uv][cyo * 8 + cxo] - pv, l);
            if (l == 0) cb.cdcin[uv][cb4] = c;
            int cc;
            unsigned nz = lane_quant(c, l, qpc, cqp_const, true, lev, cdq, cc);
            if (l == 0) { cb.cbcost[uv][cb4] = cc; cb.cbnz[uv][cb4] = nz != 0; }
        }
    }
    __syncthreads();
    if (act && !skipped && t < 2) {                    // the 2x2 DC of component t (dct_chroma)
        const int qp_per = qpc / 6, qp_rem = qpc % 6;
        const int *m = cb.cdcin[t];
        const int m1[4] = {m[0] + m[1] + m[2] + m[3], m[0] - m[1] + m[2] - m[3], m[0] + m[1] - m[2] - m[3], m[0] - m[1] - m[2] + m[3]};
        int dcnz = 0;
        for (int k = 0; k < 4; k++) {
            const int level = (abs(m1[k]) * c_q3[qp_rem][0] + 2 * cqp_const) >> (cq_bits + 1);
            if (level) dcnz = 1;
            cb.cdc[t][k] = (int16_t)isign(level, m1[k]);
        }
        const int c0 = cb.cdc[t][0], c1 = cb.cdc[t][1], c2 = cb.cdc[t][2], c3 = cb.cdc[t][3];
        const int fv[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
        const int v00 = c_dq3[qp_rem][0];
        for (int k = 0; k < 4; k++) cb.cdcq[t][k] = (fv[k] * 16 * v00 * (1 << qp_per)) >> 5;   // 8.5.11.2
        const int cost = cb.cbcost[t][0] + cb.cbcost[t][1] + cb.cbcost[t][2] + cb.cbcost[t][3];
        const int acany = cb.cbnz[t][0] | cb.cbnz[t][1] | cb.cbnz[t][2] | cb.cbnz[t][3];
        cb.creset[t] = cost < 4;                       // _CHROMA_COEFF_COST_
        cb.cdcnz[t] = (dcnz ? 1 : 0) | (acany && cost >= 4 ? 2 : 0);
    }
    __syncthreads();
    int e2 = 0;
    if (act) {
        int rv = pv;
        if (!skipped) {
            if (cb.creset[uv]) { cdq = 0; lev = 0; }
            if (l == 0) cdq = cb.cdcq[uv][cb4];
            rv = lane_inv4x4(cdq, l, pv, maxv);
        }
        out->ac[uv][cb4][l] = (int16_t)(skipped ? 0 : lev);
        out->rec[uv][cyo * 8 + cxo] = (pel)rv;
        const int e = orgc[uv][cyo * 8 + cxo] - rv;
        e2 = e * e;
        if (t < 8) out->dc[t >> 2][t & 3] = skipped ? 0 : cb.cdc[t >> 2][t & 3];
        if (t == 0) {
            int cr = 0;
            if (!skipped)
                for (int k = 0; k < 2; k++) {
                    if (cb.cdcnz[k] & 1) cr = max(cr, 1);
                    if (cb.cdcnz[k] & 2) cr = 2;
                }
            out->cbpc = cr;
        }
    }
    e2 = wave_sum(e2);
    if ((t & 63) == 0) cb.red[uv] = e2;
    __syncthreads();
    return cb.red[0] + cb.red[1];
}

// ======================================================================================
//  role "inter": the searches, P8x8 by RDCost_for_8x8blocks, the inter candidates
// ======================================================================================
template <class pel>
struct RdoInterS {
    EpzS<pel> e;                  // the motion searches (wave 0)
    alignas(4) pel orgc[2][64];
    alignas(4) uint8_t st0[JMR_NCTX];      // the slice's coding state at the MB start
    alignas(4) uint8_t strun[JMR_NCTX];    // the P8x8 running state (decided 8x8 blocks)
    alignas(4) uint8_t stc[4][JMR_NCTX];   // per sub-mode rate lane
    jmr_mbinfo nbA, nbB;
    int hasA, hasB;
    jmr_cur currun, curc[4];
    int16_t lev8[4][4][16];       // per sub-mode: the 8x8 block's four 4x4 levels (coding order)
    int16_t mvd8[4][4][2];
    pel pred8[4][64], rec8[4][64];
    int cost8[4], cbp8[4], blk8[4], dist8[4], bits8[4];
    uint32_t rgc[4], rg0, rgrun;
    int best8x8, sel;
    alignas(4) pel p8pred[256], p8rec[256];   // the P8x8 candidate, assembled block by block
    int16_t p8lev[16][16];
    int p8cbp, p8blk, p8cnt;
    int16_t fmv[2][16][2];        // MVs of the candidate(s) being coded
    int bcost[16], bnz[16], red[4];
    ChromaBuf cb[2];
    int skipx, skipy;
};

// LumaResidualCoding [J] of an inter candidate (4x4 transform) on 256 threads: MC of s.fmv[0],
// LumaResidualCoding8x8's _LUMA_COEFF_COST_ zeroing and the macroblock one; skipped: prediction only
template <class pel>
__device__ __forceinline__ void luma_inter(const DevParams &d, RdoInterS<pel> &s, RdoLuma<pel> *L, bool skipped, int mbx, int mby, int tid) {
    const int blk = tid >> 4, l = tid & 15, px4 = 4 * (blk & 3) + (l & 3), py4 = 4 * (blk >> 2) + (l >> 2);
    const int qp = d.qp + d.qpbd, maxv = d.maxv;
    const pel *refY = spl<pel>(d.refY);
    const int p = qpel_direct(refY, d.W, d.H, 4 * (16 * mbx + px4) + s.fmv[0][blk][0], 4 * (16 * mby + py4) + s.fmv[0][blk][1], maxv);
    const int org = s.e.org[py4 * 16 + px4];
    int lev = 0, rv = p, cbp = 0, cbp_blk = 0;
    if (!skipped) {
        const int c = lane_fwd4x4(org - p, l);
        int dq, cc;
        unsigned nz = lane_quant(c, l, qp, q_round(d.qsel, 15 + qp / 6), false, lev, dq, cc);
        rv = lane_inv4x4(dq, l, p, maxv);
        if (l == 0) { s.bcost[blk] = cc; s.bnz[blk] = nz != 0; }
        __syncthreads();
        int sum_cnt = 0, keep8 = 0;
        for (int b8 = 0; b8 < 4; b8++) {
            const int base = (b8 >> 1) * 8 + (b8 & 1) * 2;
            int c8 = s.bcost[base] + s.bcost[base + 1] + s.bcost[base + 4] + s.bcost[base + 5];
            const int nz8 = s.bnz[base] | s.bnz[base + 1] | s.bnz[base + 4] | s.bnz[base + 5];
            if (c8 <= 4) c8 = 0;                                   // _LUMA_COEFF_COST_
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
        if (sum_cnt <= 5) { keep8 = 0; cbp = 0; cbp_blk = 0; }      // _LUMA_MB_COEFF_COST_
        const bool keep = (keep8 >> (((blk >> 3) << 1) + ((blk & 3) >> 1))) & 1;
        if (!keep) { lev = 0; rv = p; }
    }
    L->luma[blk][l] = (int16_t)lev;
    L->rec[py4 * 16 + px4] = (pel)rv;
    const int e = org - rv;
    const int dist = block_sum(e * e, s.red, tid);
    if (tid == 0) { L->cbp = cbp; L->cbp_blk = cbp_blk; L->dist = dist; L->i16mode = 0; }
}

template <class pel>
__device__ __forceinline__ void rdo_inter_mb(const DevParams &d, RdoInterS<pel> &s, RdoScr<pel> *scr, int mbx, int mby, int tid) {
    const int wave = tid >> 6, lane = tid & 63, a = mby * d.mbw + mbx;
    const int pix_x = 16 * mbx, pix_y = 16 * mby, qp = d.qp + d.qpbd, maxv = d.maxv;
    const MbAvail mav = mb_avail(d, mbx, mby);
    // ---- inputs: the searches' (wave 0), chroma, the coding state, the neighbours' records
    EWin<pel> wn{};
    if (wave == 0) wn = epzs_load_mb(d, s.e, mbx, mby, lane);
    else if (wave == 1 || wave == 2) {
        const int t = tid - 64, uv = t >> 6, k = t & 63;
        s.orgc[uv][k] = spl<pel>(uv ? d.orgV : d.orgU)[(8 * mby + (k >> 3)) * d.Wc + 8 * mbx + (k & 7)];
    } else {
        const uint32_t rg = rdo_state_load(d, a, s.st0, tid - 192, 64);
        if (tid == 192) s.rg0 = rg;
        rdo_nb_load(d, mbx, mby, s.nbA, s.nbB, s.hasA, s.hasB, tid - 192);
    }
    __syncthreads();
    const jmr_mbinfo *A = s.hasA ? &s.nbA : nullptr, *B = s.hasB ? &s.nbB : nullptr;
    // ---- motion estimation for 16x16, 16x8, 8x16 (PartitionMotionSearch [J])
    if (wave == 0) {
        epzs_block<1>(d, s.e, wn, 0, 0, 0, 0, 0, false);
        epzs_block<2>(d, s.e, wn, 0, 0, 0, 0, 0, false);
        epzs_block<2>(d, s.e, wn, 0, 2, 1, 0, 0, false);
        epzs_block<3>(d, s.e, wn, 0, 0, 0, 0, 0, false);
        epzs_block<3>(d, s.e, wn, 2, 0, 1, 0, 0, false);
    }
    const bool p8 = inter_on(d.isr, 4) || inter_on(d.isr, 5) || inter_on(d.isr, 6) || inter_on(d.isr, 7);
    if (tid < JMR_NCTX / 4) reinterpret_cast<uint32_t *>(s.strun)[tid] = reinterpret_cast<const uint32_t *>(s.st0)[tid];
    if (tid == 0) {
        s.rgrun = s.rg0;
        memset(&s.currun, 0, sizeof(s.currun));
        s.best8x8 = 0; s.p8cbp = 0; s.p8blk = 0; s.p8cnt = 0;
    }
    __syncthreads();
    // ---- P8x8: per 8x8 block the sub-modes' searches (wave 0), their LumaResidualCoding8x8 (wave
    //      w = sub-mode 4 + w), their RDCost_for_8x8blocks rates (lane 0 of wave w), the decision
    for (int b8 = 0; b8 < 4 && p8; b8++) {
        const int X = 2 * (b8 & 1), Y = 2 * (b8 >> 1), best8x8 = s.best8x8;
        if (wave == 0) {
            epzs_block<4>(d, s.e, wn, X, Y, b8, b8, best8x8, false);
            epzs_block<5>(d, s.e, wn, X, Y, b8, b8, best8x8, false);
            epzs_block<5>(d, s.e, wn, X, Y + 1, b8, b8, best8x8, false);
            epzs_block<6>(d, s.e, wn, X, Y, b8, b8, best8x8, false);
            epzs_block<6>(d, s.e, wn, X + 1, Y, b8, b8, best8x8, false);
            epzs_block<7>(d, s.e, wn, X, Y, b8, b8, best8x8, false);
            epzs_block<7>(d, s.e, wn, X + 1, Y, b8, b8, best8x8, false);
            epzs_block<7>(d, s.e, wn, X, Y + 1, b8, b8, best8x8, false);
            epzs_block<7>(d, s.e, wn, X + 1, Y + 1, b8, b8, best8x8, false);
        }
        __syncthreads();
        const int sm = 4 + wave, b4 = lane >> 4, l = lane & 15;
        const int bx4 = X + (b4 & 1), by4 = Y + (b4 >> 1), k = by4 * 4 + bx4;
        const int px = 4 * bx4 + (l & 3), py = 4 * by4 + (l >> 2), q8 = (4 * (b4 >> 1) + (l >> 2)) * 8 + 4 * (b4 & 1) + (l & 3);
        if (inter_on(d.isr, sm)) {                      // wave-uniform
            const int p = qpel_direct(spl<pel>(d.refY), d.W, d.H, 4 * (pix_x + px) + s.e.all_mv[sm][k][0], 4 * (pix_y + py) + s.e.all_mv[sm][k][1],
                                      maxv);
            const int org = s.e.org[py * 16 + px];
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
            s.lev8[wave][b4][l] = (int16_t)lev;
            s.pred8[wave][q8] = (pel)p;
            s.rec8[wave][q8] = (pel)rv;
            const int e = org - rv;
            const int dist = wave_sum(e * e);
            if (lane == 0) { s.cost8[wave] = cost; s.cbp8[wave] = cost > 0; s.blk8[wave] = blk; s.dist8[wave] = dist; }
            if (lane < 4) {
                const int kk = (Y + (lane >> 1)) * 4 + X + (lane & 1);
                s.mvd8[wave][lane][0] = (int16_t)(s.e.all_mv[sm][kk][0] - s.e.pmv[sm][kk][0]);
                s.mvd8[wave][lane][1] = (int16_t)(s.e.all_mv[sm][kk][1] - s.e.pmv[sm][kk][1]);
            }
        }
        __syncthreads();
        if (lane == 0 && inter_on(d.isr, sm)) {         // RDCost_for_8x8blocks' rate
            copy_ctx(s.stc[wave], s.strun);
            jmr_eng e = {s.stc[wave], s.rgrun, 0};
            s.curc[wave] = s.currun;
            jmr_b8(&e, A, B, &s.curc[wave], b8, sm, (const int16_t(*)[2])s.mvd8[wave], s.cost8[wave] > 0, (const int16_t(*)[16])s.lev8[wave]);
            s.bits8[wave] = e.bits;
            s.rgc[wave] = e.range;
        }
        __syncthreads();
        if (tid == 0) {
            double best = 1e30;
            int bm = 0;
            for (int w = 0; w < 4; w++)
                if (inter_on(d.isr, 4 + w)) {
                    const double rd = rd_cost(s.dist8[w], s.bits8[w], d.lambda_rd);
                    if (rd < best) { best = rd; bm = w; }
                }
            s.sel = bm;
            s.best8x8 |= (4 + bm) << (4 * b8);
            s.rgrun = s.rgc[bm];
            s.currun = s.curc[bm];
            if (s.cost8[bm]) { s.p8cbp |= s.cbp8[bm] << b8; s.p8blk |= s.blk8[bm]; s.p8cnt += s.cost8[bm]; }
        }
        __syncthreads();
        const int sel = s.sel;
        if (tid < JMR_NCTX / 4) reinterpret_cast<uint32_t *>(s.strun)[tid] = reinterpret_cast<const uint32_t *>(s.stc[sel])[tid];
        if (tid < 64) {                                 // the decided block into the P8x8 candidate
            const int yy = tid >> 3, xx = tid & 7;
            s.p8pred[(8 * (b8 >> 1) + yy) * 16 + 8 * (b8 & 1) + xx] = s.pred8[sel][tid];
            s.p8rec[(8 * (b8 >> 1) + yy) * 16 + 8 * (b8 & 1) + xx] = s.rec8[sel][tid];
            const int qb = tid >> 4, kk = (Y + (qb >> 1)) * 4 + X + (qb & 1);
            s.p8lev[kk][tid & 15] = s.lev8[sel][qb][tid & 15];
        }
        __syncthreads();
    }
    RdoLuma<pel> *L = scr->L;
    if (p8) {                                           // SetCoeffAndReconstruction8x8
        const bool zero = s.p8cnt <= 5;                 // _LUMA_MB_COEFF_COST_
        const int blk = tid >> 4, l = tid & 15, b8 = ((blk >> 3) << 1) + ((blk & 3) >> 1), sm = (s.best8x8 >> (4 * b8)) & 15;
        const pel rv = zero ? s.p8pred[tid] : s.p8rec[tid];
        L[4].rec[tid] = rv;
        L[4].luma[blk][l] = zero ? 0 : s.p8lev[blk][l];
        if (tid < 32) {
            const int kk = tid >> 1, c = tid & 1, smk = (s.best8x8 >> (4 * (((kk >> 3) << 1) + ((kk & 3) >> 1)))) & 15;
            L[4].mv[kk][c] = s.e.all_mv[smk][kk][c];
            L[4].mvd[kk][c] = (int16_t)(s.e.all_mv[smk][kk][c] - s.e.pmv[smk][kk][c]);
        }
        if (tid < 4) L[4].b8mode[tid] = (int8_t)((s.best8x8 >> (4 * tid)) & 15);
        (void)sm;
        const int e = (int)s.e.org[tid] - (int)rv;
        const int dist = block_sum(e * e, s.red, tid);
        if (tid == 0) { L[4].cbp = zero ? 0 : s.p8cbp; L[4].cbp_blk = zero ? 0 : s.p8blk; L[4].dist = dist; L[4].i16mode = 0; }
    }
    // ---- FindSkipModeMotionVector [J], the spatial memory of the next MB (its EPZS predictor 34)
    if (tid == 0) {
        int pcx, pcy;
        set_mvp(NbBorder{s.e.bd}, 0, 0, 16, 16, pcx, pcy);
        NbBorder nbv{s.e.bd};
        int ra = -1, ax = 0, ay = 0, rb = -1, bx = 0, by = 0;
        const bool aa = nbv(-1, 0, ra, ax, ay), ab = nbv(0, -1, rb, bx, by);
        const bool zl = !aa || (ra == 0 && ax == 0 && ay == 0), za = !ab || (rb == 0 && bx == 0 && by == 0);
        s.skipx = (za || zl) ? 0 : pcx;
        s.skipy = (za || zl) ? 0 : pcy;
    }
    MbScratch *ms = d.scr + a;
    for (int i = tid; i < 7 * 32; i += NT) {
        const int m = 1 + i / 32, k = (i & 31) >> 1, c = i & 1;
        ms->all_mv[m][k][c] = s.e.all_mv[m][k][c];
    }
    __syncthreads();
    // ---- the skip / 16x16 / 16x8 / 8x16 candidates (LumaResidualCoding)
    for (int c = 0; c < 4; c++) {
        if (c > 0 && !inter_on(d.isr, c)) continue;     // uniform
        if (tid < 32) {
            const int k = tid >> 1, cc = tid & 1;
            const int v = c == 0 ? (cc ? s.skipy : s.skipx) : s.e.all_mv[c][k][cc];
            s.fmv[0][k][cc] = (int16_t)v;
            L[c].mv[k][cc] = (int16_t)v;
            L[c].mvd[k][cc] = (int16_t)(c == 0 ? 0 : v - s.e.pmv[c][k][cc]);
        }
        if (tid < 4) L[c].b8mode[tid] = (int8_t)c;
        __syncthreads();
        luma_inter(d, s, &L[c], c == 0, mbx, mby, tid);
        __syncthreads();
    }
    // ---- their chroma (ChromaResidualCoding [J], the MC of each candidate's MVs), two at a time
    for (int c0 = 0; c0 < 5; c0 += 2) {
        const int half = tid >> 7, c = c0 + half;
        const bool act = c < 5 && (c == 0 || (c == 4 ? p8 : inter_on(d.isr, c)));
        if (act && (tid & 127) < 32) {
            const int k = (tid & 127) >> 1, cc = tid & 1;
            s.fmv[half][k][cc] = L[c].mv[k][cc];
        }
        __syncthreads();
        const int dist = chroma_cand<pel>(d, s.orgc, nullptr, 0, s.fmv[half], c == 0, act, s.cb[half], act ? &scr->C[c] : nullptr, tid & 127,
                                          mbx, mby, mav.T, mav.L);
        if (act && (tid & 127) == 0) scr->C[c].dist = dist;
        __syncthreads();
    }
}

// ======================================================================================
//  role "intra": Intra16x16, the chroma intra modes, Intra4x4 by RDCost_for_4x4IntraBlocks
// ======================================================================================
template <class pel>
struct RdoIntraS {
    alignas(4) pel org[256];
    alignas(4) pel rec[256];      // the Intra4x4 reconstruction in progress
    IntraNb<pel> nb;
    Border bd;
    int8_t ipred_cur[16];
    alignas(4) uint8_t st0[JMR_NCTX];
    alignas(4) uint8_t stc[9][JMR_NCTX];
    jmr_mbinfo nbA, nbB;
    int hasA, hasB;
    uint32_t rg0;
    int P[13];
    int16_t lev[9][16];
    pel r4[9][16];
    int dist[9], bits[9], nz[9];
    int mpm, sel, i16mode, i16cost;
    int i4cbp, i4blk;
    int dc[16], dcdq[16], bnz[16], red[4];
    int16_t dclev[16];
    ChromaBuf cb[2];
};

template <class pel>
__device__ __forceinline__ int i4_lpix(const RdoIntraS<pel> &s, int x, int y) {
    if (y < 0) return s.nb.rtop[x + 1];
    if (x < 0) return s.nb.rleft[y];
    return s.rec[16 * y + x];
}

template <class pel>
__device__ __forceinline__ void rdo_intra_mb(const DevParams &d, RdoIntraS<pel> &s, RdoScr<pel> *scr, int mbx, int mby, int tid) {
    const int wave = tid >> 6, lane = tid & 63, a = mby * d.mbw + mbx;
    const int W = d.W, pix_x = 16 * mbx, pix_y = 16 * mby, qp = d.qp + d.qpbd, maxv = d.maxv;
    const MbAvail mav = mb_avail(d, mbx, mby);
    const bool avL = mav.L, avT = mav.T, avTL = mav.TL, avTR = mav.TR;
    const pel *orgY = spl<pel>(d.orgY);
    s.org[tid] = orgY[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)];
    if (tid < 128) load_orgc(d, s.nb, tid, mbx, mby);
    else if (tid < 128 + 71) load_intra_nb(d, s.nb, tid - 128, mbx, mby);
    else if (tid >= 208 && tid < 218) load_border(d, s.bd, tid - 208, mbx, mby);
    if (tid >= 192) {
        const uint32_t rg = rdo_state_load(d, a, s.st0, tid - 192, 64);
        if (tid == 192) s.rg0 = rg;
        rdo_nb_load(d, mbx, mby, s.nbA, s.nbB, s.hasA, s.hasB, tid - 192);
    }
    __syncthreads();
    const jmr_mbinfo *A = s.hasA ? &s.nbA : nullptr, *B = s.hasB ? &s.nbB : nullptr;
    RdoLuma<pel> *L = scr->L;
    // ---- Intra16x16: the find_sad_16x16 mode (wave 0), dct_luma_16x16 on every thread
    if (wave == 0) {
        int c16, m16;
        i16_pick(d, s.org, s.nb, lane, avL, avT, avTL, c16, m16);
        if (lane == 0) { s.i16mode = m16; s.i16cost = c16; }
    }
    __syncthreads();
    {
        const int blk = tid >> 4, l = tid & 15, px4 = 4 * (blk & 3) + (l & 3), py4 = 4 * (blk >> 2) + (l >> 2);
        const pel *T = s.nb.rtop + 1, *Lf = s.nb.rleft;
        const I16Par par = i16_params(T, Lf, avT, avL, (maxv + 1) >> 1);
        const int p = i16_pred(par, T, Lf, s.i16mode, px4, py4, maxv);
        int lev, rv;
        i16_code(p, (int)s.org[py4 * 16 + px4], qp, q_round(q_sel16(d.qsel), 15 + qp / 6), s.dc, s.dcdq, s.dclev, s.bnz, tid, maxv, lev, rv);
        L[5].luma[blk][l] = (int16_t)lev;
        L[5].rec[py4 * 16 + px4] = (pel)rv;
        if (tid < 16) L[5].luma_dc[tid] = s.dclev[tid];
        const int e = (int)s.org[py4 * 16 + px4] - rv;
        const int dist = block_sum(e * e, s.red, tid);   // (synchronises: bnz final)
        if (tid == 0) {
            int cbp = 0, blkm = 0;
            for (int b = 0; b < 16; b++)
                if (s.bnz[b]) { cbp = 15; blkm |= 1 << b; }
            L[5].cbp = cbp; L[5].cbp_blk = blkm; L[5].dist = dist; L[5].i16mode = s.i16mode;
        }
        if (tid < 32) L[5].mv[tid >> 1][tid & 1] = 0;
    }
    // ---- the four chroma intra modes (ChromaResidualCoding of IntraChromaPrediction8x8 [J])
    const bool cav[4] = {true, avL, avT, avT && avL && avTL};
    for (int m0 = 0; m0 < 4; m0 += 2) {
        const int half = tid >> 7, m = m0 + half;
        const bool act = m == 0 || (m == 1 ? avL : m == 2 ? avT : cav[3]);
        const int dist = chroma_cand<pel>(d, s.nb.orgc, &s.nb, m, nullptr, false, act, s.cb[half], act ? &scr->C[5 + m] : nullptr, tid & 127,
                                          mbx, mby, avT, avL);
        if (act && (tid & 127) == 0) scr->C[5 + m].dist = dist;
        __syncthreads();
    }
    // ---- Intra4x4: Mode_Decision_for_4x4IntraBlocks [J] by RDCost_for_4x4IntraBlocks, 16 blocks in
    //      coding order: 9 modes x 16 lanes code, lane 16 m rates mode m, thread 0 decides
    if (tid == 0) { s.i4cbp = 0; s.i4blk = 0; }
    const int rnd = q_round(d.qsel, 15 + qp / 6);
    for (int i = 0; i < 16; i++) {
        const int b8 = i >> 2, b4 = i & 3;
        const int bx = 8 * (b8 & 1) + 4 * (b4 & 1), by = 8 * (b8 >> 1) + 4 * (b4 >> 1), bx4 = bx >> 2, by4 = by >> 2, blk = 4 * by4 + bx4;
        const bool up = by > 0 || avT, left = bx > 0 || avL;
        const bool ul = (bx > 0 && by > 0) || (bx == 0 && by > 0 && avL) || (bx > 0 && by == 0 && avT) || (bx == 0 && by == 0 && avTL);
        bool ur = by == 0 ? (bx + 4 <= 15 ? avT : avTR) : (bx + 4 <= 15);
        if ((bx == 4 || bx == 12) && (by == 4 || by == 12)) ur = false;
        if (tid < 13) {
            int v;
            if (tid == 0) v = ul ? i4_lpix(s, bx - 1, by - 1) : 0;
            else if (tid <= 4) v = up ? i4_lpix(s, bx + tid - 1, by - 1) : 0;
            else if (tid <= 8) v = up ? i4_lpix(s, ur ? bx + tid - 1 : bx + 3, by - 1) : 0;
            else v = left ? i4_lpix(s, bx - 1, by + tid - 9) : 0;
            s.P[tid] = v;
        } else if (tid == 64) {
            const int upM = by > 0 ? s.ipred_cur[blk - 4] : s.bd.ipm[1 + bx4];
            const int leftM = bx > 0 ? s.ipred_cur[blk - 1] : s.bd.ipm[6 + by4];
            s.mpm = (upM < 0 || leftM < 0) ? 2 : min(upM, leftM);
        }
        __syncthreads();
        const int m = tid >> 4, l = tid & 15;
        const bool avm = m < 9 && (m == 2 || ((m == 0 || m == 3 || m == 7) && up) || ((m == 1 || m == 8) && left) || (up && left && ul));
        if (m < 9) {                                    // 144 threads: the nine modes' dct_luma
            const int e = c_i4tab[m][l], ty = e & 3;
            const int pa = s.P[(e >> 2) & 15], pb = s.P[(e >> 6) & 15], pc = s.P[(e >> 10) & 15];
            const int st = s.P[1] + s.P[2] + s.P[3] + s.P[4], sl = s.P[9] + s.P[10] + s.P[11] + s.P[12];
            const int dc = (up && left) ? (st + sl + 4) >> 3 : left ? (sl + 2) >> 2 : up ? (st + 2) >> 2 : (maxv + 1) >> 1;
            const int p = ty == 1 ? (pa + pb + 1) >> 1 : ty == 2 ? (pa + 2 * pb + pc + 2) >> 2 : dc;
            const int org = s.org[(by + (l >> 2)) * 16 + bx + (l & 3)];
            const int c = lane_fwd4x4(org - p, l);
            int lev, dq, cc;
            const unsigned nz = lane_quant(c, l, qp, rnd, false, lev, dq, cc);
            const int rv = lane_inv4x4(dq, l, p, maxv);
            s.lev[m][l] = (int16_t)lev;
            s.r4[m][l] = (pel)rv;
            const int dist = row16_sum((org - rv) * (org - rv));
            if (l == 0) { s.dist[m] = dist; s.nz[m] = nz != 0; }
        }
        __syncthreads();
        if (l == 0 && avm) {                            // lane 16 m: the block's rate in mode m
            copy_ctx(s.stc[m], s.st0);
            jmr_eng e = {s.stc[m], s.rg0, 0};
            const int mpm = s.mpm;
            jmr_i4(&e, A, B, bx4, by4, m == mpm ? -1 : m < mpm ? m : m - 1, s.lev[m]);
            s.bits[m] = e.bits;
        }
        __syncthreads();
        if (tid == 0) {
            double best = 1e30;
            int bm = 2;
            for (int mm = 0; mm < 9; mm++) {
                const bool av = mm == 2 || ((mm == 0 || mm == 3 || mm == 7) && up) || ((mm == 1 || mm == 8) && left) || (up && left && ul);
                if (!av) continue;
                const double rd = rd_cost(s.dist[mm], s.bits[mm], d.lambda_rd);
                if (rd < best) { best = rd; bm = mm; }
            }
            s.sel = bm;
            s.ipred_cur[blk] = (int8_t)bm;
            const int mpm = s.mpm;
            L[6].imode[blk] = (int8_t)bm;
            L[6].ipm[blk] = (int8_t)(bm == mpm ? -1 : bm < mpm ? bm : bm - 1);
            if (s.nz[bm]) { s.i4cbp |= 1 << b8; s.i4blk |= 1 << blk; }
        }
        __syncthreads();
        if (tid < 16) {
            const int sel = s.sel;
            s.rec[(by + (tid >> 2)) * 16 + bx + (tid & 3)] = s.r4[sel][tid];
            L[6].luma[blk][tid] = s.lev[sel][tid];
        }
        __syncthreads();
    }
    L[6].rec[tid] = s.rec[tid];
    const int e = (int)s.org[tid] - (int)s.rec[tid];
    const int dist = block_sum(e * e, s.red, tid);
    if (tid == 0) { L[6].cbp = s.i4cbp; L[6].cbp_blk = s.i4blk; L[6].dist = dist; L[6].i16mode = 0; }
    if (tid < 32) L[6].mv[tid >> 1][tid & 1] = 0;
}

template <class pel>
__global__ __launch_bounds__(NT, 2) void k_rdo_analyse(const TickArgs t) {
    __shared__ union {
        RdoInterS<pel> in;
        RdoIntraS<pel> ia;
    } s;
    const int tid = threadIdx.x, nP = t.pre[t.nP], nPg = xcd_grid(nP), tot = t.pre[t.npic], b = blockIdx.x;
    RdoScr<pel> *base = reinterpret_cast<RdoScr<pel> *>(t.rscr);
    if (b < nPg) {
        const int m = xcd_block(b, nP);
        if (m >= nP) return;                            // padding block (whole workgroup)
        const int e = tick_entry(t, m);
        const DevParams d = tick_params(t, e);
        int mbx, mby;
        tick_mb(t, d, e, m, mbx, mby);
        rdo_inter_mb(d, s.in, base + m, mbx, mby, tid);
    } else {
        const int m = xcd_block(b - nPg, tot);
        if (m >= tot) return;
        const int e = tick_entry(t, m);
        const DevParams d = tick_params(t, e);
        int mbx, mby;
        tick_mb(t, d, e, m, mbx, mby);
        rdo_intra_mb(d, s.ia, base + m, mbx, mby, tid);
    }
}

// ======================================================================================
//  k_rdo_final: RDCost_for_macroblocks over the candidates, the decision, its outputs
// ======================================================================================
template <class pel>
struct RdoFinS {
    alignas(4) uint8_t st0[JMR_NCTX];
    alignas(4) uint8_t stc[RD_NCAND][JMR_NCTX];
    jmr_mbinfo nbA, nbB, out[RD_NCAND];
    int hasA, hasB;
    uint32_t rg0, rgo[RD_NCAND];
    double rd[RD_NCAND];
    int bits[RD_NCAND], ci[RD_NCAND], ccm[RD_NCAND];
    int ncand, win;
    alignas(4) pel rec[256];
    pel cfin[2][64];
    int16_t fmv[16][2];
    DbkS<pel> db;
};

template <class pel>
__global__ __launch_bounds__(NT) void k_rdo_final(const TickArgs t) {
    __shared__ RdoFinS<pel> s;
    const int tid = threadIdx.x, tot = t.pre[t.npic];
    const int m = xcd_block(blockIdx.x, tot);
    if (m >= tot) return;
    const int e = tick_entry(t, m);
    const DevParams d = tick_params(t, e);
    int mbx, mby;
    tick_mb(t, d, e, m, mbx, mby);
    const RdoScr<pel> *scr = reinterpret_cast<const RdoScr<pel> *>(t.rscr) + m;
    const int a = mby * d.mbw + mbx, W = d.W, Wc = d.Wc, W4 = d.W >> 2, pix_x = 16 * mbx, pix_y = 16 * mby;
    const bool slice_p = d.slice_type == JMH_P_SLICE;
    const MbAvail mav = mb_avail(d, mbx, mby);
    if (tid < 64) {
        const uint32_t rg = rdo_state_load(d, a, s.st0, tid, 64);
        if (tid == 0) s.rg0 = rg;
    } else if (tid < 128) rdo_nb_load(d, mbx, mby, s.nbA, s.nbB, s.hasA, s.hasB, tid - 64);
    else if (tid == 128) {                              // the candidates in JM's order
        const bool p8 = inter_on(d.isr, 4) || inter_on(d.isr, 5) || inter_on(d.isr, 6) || inter_on(d.isr, 7);
        const bool cav[4] = {true, mav.L, mav.T, mav.T && mav.L && mav.TL};
        int n = 0;
        for (int cm = 0; cm < 4; cm++) {
            if (!cav[cm]) continue;
            for (int i = 0; i < RD_NL; i++) {
                const bool valid = i >= 5 || (slice_p && (i == 0 || (i == 4 ? p8 : inter_on(d.isr, i))));
                if (!valid || (cm != 0 && i < 5)) continue;
                s.ci[n] = i; s.ccm[n] = cm; n++;
            }
        }
        s.ncand = n;
    }
    __syncthreads();
    const jmr_mbinfo *A = s.hasA ? &s.nbA : nullptr, *B = s.hasB ? &s.nbB : nullptr;
    // ---- one lane per candidate: its rate on its own copy of the coding state
    if (tid < s.ncand) {
        const int i = s.ci[tid], cm = s.ccm[tid];
        const RdoLuma<pel> &L = scr->L[i];
        const RdoChroma<pel> &C = scr->C[i >= 5 ? 5 + cm : i];
        copy_ctx(s.stc[tid], s.st0);
        jmr_eng en = {s.stc[tid], s.rg0, 0};
        if (i == 0) jmr_skip(&en, A, B, &s.out[tid]);
        else {
            jmr_cand r;
            r.mb_type = i == 4 ? JMH_P8x8 : i == 5 ? JMH_I16MB : i == 6 ? JMH_I4MB : i;
            r.cbp = L.cbp | C.cbpc << 4;
            r.i16mode = L.i16mode;
            r.cmode = i >= 5 ? cm : 0;
            r.t8 = 0;
            for (int q = 0; q < 4; q++) r.b8mode[q] = L.b8mode[q];
            r.ipm = L.ipm;
            r.mvd = L.mvd;
            r.luma = L.luma;
            r.luma_dc = L.luma_dc;
            r.cdc = C.dc;
            r.cac = C.ac;
            jmr_mb(&en, A, B, &r, slice_p, 0, &s.out[tid]);
        }
        s.bits[tid] = en.bits;
        s.rgo[tid] = en.range;
        s.rd[tid] = rd_cost(L.dist + C.dist, en.bits, d.lambda_rd);
    }
    __syncthreads();
    if (tid == 0) {                                     // strict '<' in JM's order
        double best = 1e30;
        int w = 0;
        for (int k = 0; k < s.ncand; k++)
            if (s.rd[k] < best) { best = s.rd[k]; w = k; }
        s.win = w;
    }
    __syncthreads();
    // ---- the chosen macroblock: results, reconstruction, picture arrays, coding state
    const int w = s.win, bi = s.ci[w], bcm = s.ccm[w];
    const RdoLuma<pel> &L = scr->L[bi];
    const RdoChroma<pel> &C = scr->C[bi >= 5 ? 5 + bcm : bi];
    const bool is_intra = bi >= 5;
    const int mb_type = bi == 0 ? JMH_PSKIP : bi == 4 ? JMH_P8x8 : bi == 5 ? JMH_I16MB : bi == 6 ? JMH_I4MB : bi;
    const int cbp = L.cbp | C.cbpc << 4, cbp_blk = L.cbp_blk;
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
        res->transform_8x8 = 0; res->pad0 = 0;
        res->min_cost = s.bits[w];                      // the chosen candidate's rate (bits)
        res->reserved = 0;
    }
    const int blk = tid >> 4, l = tid & 15;
    res->luma[blk][l] = L.luma[blk][l];
    if (tid < 16) {
        const int k = tid;
        const int ip = mb_type == JMH_I4MB ? L.imode[k] : 2;
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
        if (tid < JMR_NCTX / 4) dst[tid] = reinterpret_cast<const uint32_t *>(s.stc[w])[tid];
        const int nw = (int)sizeof(jmr_mbinfo) / 4;
        if (tid >= 128 && tid < 128 + nw)
            reinterpret_cast<uint32_t *>(d.rp->mbi + a)[tid - 128] = reinterpret_cast<const uint32_t *>(&s.out[w])[tid - 128];
        if (tid == 192) {
            jmr_eng en = {nullptr, s.rgo[w], 0};
            if ((a + 1) % d.slice_mbs != 0 && a + 1 < d.mbw * d.mbh) jmr_end_of_mb(&en);
            d.rp->range[slice] = en.range;
        }
    }
    // ---- DeblockMb [J] (jmh_deblock.h)
    if (d.dbkY) {
        const int qpi = iclip(-d.qpbd, 51, d.qp + d.cqp_off), qpcy = qpi < 0 ? qpi : c_qpc[qpi];
        deblock_mb(d, s.db, s.rec, s.cfin, s.fmv, is_intra, cbp_blk, false, d.qp, qpcy, mbx, mby, tid);
    }
}

hipError_t jmh_launch_rdo(const TickArgs &t, hipStream_t st) {
    const int tot = t.pre[t.npic];
    if (!tot) return hipSuccess;
    const int na = xcd_grid(t.pre[t.nP]) + xcd_grid(tot);
    if (t.bd > 8) hipLaunchKernelGGL(k_rdo_analyse<uint16_t>, dim3(na), dim3(NT), 0, st, t);
    else hipLaunchKernelGGL(k_rdo_analyse<uint8_t>, dim3(na), dim3(NT), 0, st, t);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    if (t.bd > 8) hipLaunchKernelGGL(k_rdo_final<uint16_t>, dim3(xcd_grid(tot)), dim3(NT), 0, st, t);
    else hipLaunchKernelGGL(k_rdo_final<uint8_t>, dim3(xcd_grid(tot)), dim3(NT), 0, st, t);
    return hipGetLastError();
}
