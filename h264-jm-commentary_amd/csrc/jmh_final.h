// jmh_final.h — the second half of encode_one_macroblock [J] (RDO off) for one macroblock on 256
// threads: the mode decision over the analysis costs, then the residual coding of the chosen mode
// with 16-lane transform groups (LumaResidualCoding / dct_luma_16x16 / dct_chroma +
// reconstruction), or, with Transform8x8Mode, TransformDecision and dct_luma8x8 on one wave per
// 8x8 block, the outputs the next diagonal depends on (reconstruction, MVs, reference indices,
// intra modes) and the fused DeblockMb, run by k_mb_final (jmh_final.hip).  (Round 4 also ran it
// as a last role of k_mb_analyse, waiting on per-MB flags: 1159 -> 792 MP/s on config 2,
// profiles/r7m_fused_final_ab.txt, not kept.)
#ifndef JMH_FINAL_H
#define JMH_FINAL_H
#include "jmh_deblock.h"
#include "jmh_intra.h"

// pel: uint8_t (bit depth 8) or uint16_t (High 10) samples
template <class pel>
struct FinS {
    pel org[256];
    pel orgc[2][64];
    pel rec[256];
    pel pred[256];                       // inter prediction (TransformDecision / 8x8 path)
    int tdc[4][2];                       // per 8x8: sum of 4x4 SATDs, 8x8 SATD
    pel rtop[24];                        // luma row y = -1, x = -1..19 -> [x + 1]
    pel rleft[16];
    pel ctop[2][12];                     // chroma rows y = -1, x = -1..7 -> [x + 1]
    pel cleft[2][8];
    int16_t fmv[16][2];
    int16_t lev[16][16];
    int bcost[16];
    int bnz[16];
    int dc[16];
    int dcdq[16];
    int16_t dclev[16];
    int cdcin[2][4];
    int cdcq[2][4];
    int16_t cdc[2][4];
    int16_t cac[2][4][16];
    int cbcost[2][4];
    int cbnz[2][4];
    int creset[2];
    int cdcnz[2];
    pel cfin[2][64];
    DbkS<pel> db;                        // the fused deblocking (jmh_deblock.h)
};

// OCC (k_mb_final) workgroups per CU: 8 (64 VGPRs, a few spilled) for ticks of more than 5 x 256 MBs (2160p,
// one dispatch round), 5 (no spills, a shorter per-MB chain) for smaller ticks
// T8: built with Transform8x8Mode's paths (I8MB, TransformDecision, dct_luma8x8); the
// instantiation without them folds d.t8 = 0, and 8-bit samples fold Clip1 = 255, QpBdOffset = 0
// NTH: threads of the workgroup.  256: the luma coding on all of them, the chroma coding after it on
// threads 0..127.  512 (k_mb_final512, k_mb_flow): luma on threads 0..255 while waves 4 and 5 run the
// chroma prediction, transform and quantisation (dct_chroma's first half) beside it; only the
// chroma DC and the inverse transform follow the luma.  Every thread of the workgroup calls it.
// mc(X, Y): the luma sample at quarter-pel position (X, Y) of the reference (qpel_direct from HBM in
// the tick kernels; k_mb_flow reads its search window's G / b / h / j planes in LDS).  porg / pnb:
// the MB's source and intra neighbourhood already in LDS (k_mb_flow's analysis state), or null:
// loaded here.
template <int OCC, class pel, bool T8, int NTH, class MC>
__device__ __forceinline__ void final_core(DevParams d, FinS<pel> &s, int mbx, int mby, int tid, MC mc, const pel *porg = nullptr,
                                           const IntraNb<pel> *pnb = nullptr) {
    constexpr bool W2 = NTH == 512;
    static_assert(NTH == 256 || NTH == 512, "final_core runs on 256 or 512 threads");
    if constexpr (!T8) d.t8 = 0;
    if constexpr (sizeof(pel) == 1) { d.maxv = 255; d.qpbd = 0; }
    const bool lu = !W2 || tid < 256;                    // luma threads (wave-uniform)
    const int ct = W2 ? tid - 256 : tid;                 // chroma thread index (valid in [0, 128))
    const bool chv = ct >= 0 && ct < 128;
    const int pix_x = 16 * mbx, pix_y = 16 * mby;
    const int W = d.W, Wc = d.Wc, W4 = d.W >> 2;
    const int slice_p = d.slice_type == JMH_P_SLICE;
    // QPY (deblocking) and QP'Y = QPY + QpBdOffsetY (quantisation); Clip1 to maxv
    const int qpy = d.qp, qp = d.qp + d.qpbd, maxv = d.maxv;
    const pel *orgY = spl<pel>(d.orgY), *orgU = spl<pel>(d.orgU), *orgV = spl<pel>(d.orgV);
    const pel *refU = spl<pel>(d.refU), *refV = spl<pel>(d.refV);
    pel *recY = spl<pel>(d.recY), *recU = spl<pel>(d.recU), *recV = spl<pel>(d.recV);
    const MbAvail mav = intra_avail(d, mbx, mby);   // (the intra prediction's neighbours)
    const bool avL = mav.L, avT = mav.T, avTL = mav.TL;
    const bool prof = prof_mb_here(d, mbx, mby);
    PSTAMP(16);
    const MbScratch *sc = d.scr + mby * d.mbw + mbx;

    // ---- inputs into LDS (unless the caller's LDS holds them)
    const pel *S_org = porg ? porg : s.org;
    const pel(*S_orgc)[64] = pnb ? pnb->orgc : s.orgc;
    const pel *S_rtop = pnb ? pnb->rtop : s.rtop, *S_rleft = pnb ? pnb->rleft : s.rleft;
    const pel(*S_ctop)[12] = pnb ? pnb->ctop : s.ctop;
    const pel(*S_cleft)[8] = pnb ? pnb->cleft : s.cleft;
    if (lu && !porg) s.org[tid] = orgY[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)];
    if (d.dbkY) deblock_prefetch<pel, NTH>(d, s.db, mbx, mby, tid);   // its latency under the decision and the luma
    if (!pnb && (!W2 || tid >= 256)) {
        const int u = ct;
        if (u < 128) {
            const int uv = u >> 6, k = u & 63;
            s.orgc[uv][k] = (uv ? orgV : orgU)[((pix_y >> 1) + (k >> 3)) * Wc + (pix_x >> 1) + (k & 7)];
        } else if (u >= 128 && u < 149) {
            const int x = u - 129;
            const bool av = x < 0 ? avTL : x < 16 ? avT : false;
            s.rtop[x + 1] = av ? recY[(pix_y - 1) * W + pix_x + x] : 0;
        } else if (u >= 160 && u < 176) {
            const int y = u - 160;
            s.rleft[y] = avL ? recY[(pix_y + y) * W + pix_x - 1] : 0;
        } else if (u >= 192 && u < 210) {
            const int i = u - 192, uv = i / 9, x = i - 9 * uv - 1;
            const bool av = x < 0 ? avTL : avT;
            s.ctop[uv][x + 1] = av ? (uv ? recV : recU)[((pix_y >> 1) - 1) * Wc + (pix_x >> 1) + x] : 0;
        } else if (u >= 224 && u < 240) {
            const int i = u - 224, uv = i >> 3, y = i & 7;
            s.cleft[uv][y] = avL ? (uv ? recV : recU)[((pix_y >> 1) + y) * Wc + (pix_x >> 1) - 1] : 0;
        }
    }

    // ---- mode decision (encode_one_macroblock, RDO off): costs from k_mb_analyse
    int min_cost = BIGCOST, best_mode = 1, best8x8 = 0;
    if (slice_p) {
        for (int mode = 1; mode < 4; mode++) {
            if (!inter_on(d.isr, mode)) continue;
            const int cost = mode == 1 ? sc->motion_cost[1][0] : sc->motion_cost[mode][0] + sc->motion_cost[mode][1];
            if (cost < min_cost) { best_mode = mode; min_cost = cost; }
        }
        if (inter_on(d.isr, 4) || inter_on(d.isr, 5) || inter_on(d.isr, 6) || inter_on(d.isr, 7)) {
            best8x8 = sc->best8x8;
            if (sc->cost8x8 < min_cost) { best_mode = JMH_P8x8; min_cost = sc->cost8x8; }
        }
    }
    if (d.t8 && sc->i8cost <= min_cost) { min_cost = sc->i8cost; best_mode = JMH_I8MB; }   // item 27
    if (sc->i4cost <= min_cost) { min_cost = sc->i4cost; best_mode = JMH_I4MB; }
    const int i16mode = sc->i16mode;
    if (sc->i16cost < min_cost) { min_cost = sc->i16cost; best_mode = JMH_I16MB; }
    const int is_intra = best_mode == JMH_I4MB || best_mode == JMH_I16MB || best_mode == JMH_I8MB;
    int b8mode[4];
    for (int b = 0; b < 4; b++)
        b8mode[b] = best_mode == JMH_P8x8 ? (best8x8 >> (4 * b)) & 15 : best_mode == JMH_I4MB ? JMH_IBLOCK : best_mode == JMH_I16MB ? 0
                  : best_mode == JMH_I8MB ? JMH_I8MB : best_mode;
    if (tid < 32) {
        const int k = tid >> 1, c = tid & 1, b8 = ((k >> 3) << 1) + ((k & 3) >> 1);
        const int bm = best_mode == JMH_P8x8 ? (best8x8 >> (4 * b8)) & 15 : best_mode;
        s.fmv[k][c] = is_intra ? 0 : sc->all_mv[bm][k][c];
    }
    __syncthreads();

    // ======== chroma prediction, ahead of the luma: the inter prediction's reference reads then
    // travel with the luma MC's instead of one round trip after them
    const int c_mode = is_intra ? sc->c_mode : 0;
    const int l = tid & 15;
    const int cuv = (ct >> 4) >> 2, cb = (ct >> 4) & 3;
    const int cxo = (cb & 1) * 4 + (ct & 3), cyo = (cb >> 1) * 4 + ((ct & 15) >> 2);
    int cpredv = 0;
    if (chv) {
        if (is_intra) {
            cpredv = chroma_pred_px(S_ctop[cuv] + 1, S_cleft[cuv], S_ctop[cuv][0], avT, avL, c_mode, cxo, cyo, maxv);
        } else {
            // OneComponentChromaPrediction4x4 [J] / 8.4.2.2.2
            const pel *R = cuv ? refV : refU;
            const int vx = s.fmv[(cyo >> 1) * 4 + (cxo >> 1)][0], vy = s.fmv[(cyo >> 1) * 4 + (cxo >> 1)][1];
            const int ii = ((pix_x >> 1) + cxo) * 8 + vx, jj = ((pix_y >> 1) + cyo) * 8 + vy;
            const int x0 = iclip(0, Wc - 1, ii >> 3), y0 = iclip(0, d.Hc - 1, jj >> 3);
            const int x1 = iclip(0, Wc - 1, (ii + 7) >> 3), y1 = iclip(0, d.Hc - 1, (jj + 7) >> 3);
            const int fx = ii & 7, fy = jj & 7;
            cpredv = ((8 - fx) * (8 - fy) * R[y0 * Wc + x0] + fx * (8 - fy) * R[y0 * Wc + x1] + (8 - fx) * fy * R[y1 * Wc + x0] +
                      fx * fy * R[y1 * Wc + x1] + 32) >> 6;
        }
    }
    // dct_chroma [J] in three parts: (A) forward transform + AC quantisation per 4x4, (B) the 2x2 DC
    // on two threads, (C) inverse transform + reconstruction.  QPc of qPI = Clip3(-QpBdOffsetC, 51,
    // QPY + chroma_qp_index_offset) (8.5.8, Table 8-15: negative qPI map to themselves), quantised
    // at QP'c = QPc + QpBdOffsetC
    const int qpi = iclip(-d.qpbd, 51, qpy + d.cqp_off), qpcy = qpi < 0 ? qpi : c_qpc[qpi], qpc = qpcy + d.qpbd;
    const int cq_bits = 15 + qpc / 6;
    const int cqp_const = q_round(d.qsel, cq_bits);
    int cdq = 0;
    auto chroma_a = [&]() {
        if (chv) {
            const int c = lane_fwd4x4(S_orgc[cuv][cyo * 8 + cxo] - cpredv, l);
            if (l == 0) s.cdcin[cuv][cb] = c;
            int lev, cc;
            unsigned nz = lane_quant(c, l, qpc, cqp_const, true, lev, cdq, cc);
            s.cac[cuv][cb][l] = (int16_t)lev;
            if (l == 0) { s.cbcost[cuv][cb] = cc; s.cbnz[cuv][cb] = nz != 0; }
        }
    };
    auto chroma_b = [&]() {
        if (ct >= 0 && ct < 2) {
            const int uv = ct, qp_per = qpc / 6, qp_rem = qpc % 6;
            const int *m = s.cdcin[uv];
            int m1[4] = {m[0] + m[1] + m[2] + m[3], m[0] - m[1] + m[2] - m[3], m[0] + m[1] - m[2] - m[3], m[0] - m[1] - m[2] + m[3]};
            int dcnz = 0;
            for (int k = 0; k < 4; k++) {
                int level = (abs(m1[k]) * c_q3[qp_rem][0] + 2 * cqp_const) >> (cq_bits + 1);
                if (level) dcnz = 1;
                s.cdc[uv][k] = (int16_t)isign(level, m1[k]);
            }
            int c0 = s.cdc[uv][0], c1 = s.cdc[uv][1], c2 = s.cdc[uv][2], c3 = s.cdc[uv][3];
            int fv[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
            int v00 = c_dq3[qp_rem][0];
            for (int k = 0; k < 4; k++) s.cdcq[uv][k] = (fv[k] * 16 * v00 * (1 << qp_per)) >> 5;   // 8.5.11.2
            int cost = s.cbcost[uv][0] + s.cbcost[uv][1] + s.cbcost[uv][2] + s.cbcost[uv][3];
            int acany = s.cbnz[uv][0] | s.cbnz[uv][1] | s.cbnz[uv][2] | s.cbnz[uv][3];
            s.creset[uv] = cost < 4;                                  // _CHROMA_COEFF_COST_
            s.cdcnz[uv] = (dcnz ? 1 : 0) | (acany && cost >= 4 ? 2 : 0);
        }
    };
    auto chroma_c = [&]() {
        if (chv) {
            if (s.creset[cuv]) { cdq = 0; s.cac[cuv][cb][l] = 0; }
            if (l == 0) cdq = s.cdcq[cuv][cb];
            s.cfin[cuv][cyo * 8 + cxo] = (pel)lane_inv4x4(cdq, l, cpredv, maxv);
        }
    };
    if constexpr (W2) chroma_a();                                      // beside the luma coding

    // ======== luma residual coding: 16 blocks x 16 lanes (threads 0..255)
    int cbp = 0, cbp_blk = 0;
    bool tr8 = false;                                                 // 8x8 transform
    const int blk = tid >> 4, lx = l & 3, ly = l >> 2;
    const int px4 = 4 * (blk & 3) + lx, py4 = 4 * (blk >> 2) + ly;   // MB pixel of this lane
    const int w8 = tid >> 6, l8 = tid & 63;                           // 8x8 layout: wave = 8x8 block
    const int qx = 8 * (w8 & 1) + (l8 & 7), qy = 8 * (w8 >> 1) + (l8 >> 3);
    if (best_mode == JMH_I8MB) {
        cbp = sc->i8cbp; tr8 = true;
        for (int b = 0; b < 4; b++)
            if ((cbp >> b) & 1) cbp_blk |= 0x33 << ((b >> 1) * 8 + (b & 1) * 2);
        if (lu) {
            s.lev[blk][l] = sc->i8lev[blk][l];
            s.rec[tid] = spl<pel>(sc->i8rec)[tid];
        }
    } else if (best_mode == JMH_I4MB) {
        cbp = sc->i4cbp; cbp_blk = sc->i4blk;
        if (lu) {
            s.lev[blk][l] = sc->i4lev[blk][l];
            s.rec[tid] = spl<pel>(sc->i4rec)[tid];
        }
    } else if (best_mode == JMH_I16MB) {
        // dct_luma_16x16 [J] (jmh_intra.h i16_code)
        int p = 0, org = 0;
        if (lu) {
            const pel *T = S_rtop + 1, *L = S_rleft;
            const I16Par par = i16_params(T, L, avT, avL, (maxv + 1) >> 1);
            p = i16_pred(par, T, L, i16mode, px4, py4, maxv);
            org = (int)S_org[py4 * 16 + px4];
        }
        int lev, rv;
        i16_code(p, org, qp, q_round(q_sel16(d.qsel), 15 + qp / 6), s.dc, s.dcdq, s.dclev, s.bnz, tid, maxv, lev, rv, lu);
        if (lu) {
            s.lev[blk][l] = (int16_t)lev;
            s.rec[py4 * 16 + px4] = (pel)rv;
        }
        __syncthreads();
        for (int b = 0; b < 16; b++)
            if (s.bnz[b]) { cbp = 15; cbp_blk |= 1 << b; }
    } else {
        // LumaResidualCoding / LumaResidualCoding8x8 (+ SetCoeffAndReconstruction8x8)
        const int p = lu ? mc(4 * (pix_x + px4) + s.fmv[blk][0], 4 * (pix_y + py4) + s.fmv[blk][1]) : 0;
        if (d.t8 && (best_mode <= 3 || best8x8 == 0x4444)) {
            // TransformDecision [J] (item 29): sum of 4x4 SATDs vs sum of 8x8 SATDs of the residual
            if (lu) s.pred[py4 * 16 + px4] = (pel)p;
            __syncthreads();
            if (lu) {
                const int dv = S_org[qy * 16 + qx] - s.pred[qy * 16 + qx];
                const int c4 = wave_satd4x4s(dv, l8, d.use_hadamard), c8 = wave_satd8(dv, l8, d.use_hadamard);
                if (l8 == 0) { s.tdc[w8][0] = c4; s.tdc[w8][1] = c8; }
            }
            __syncthreads();
            tr8 = s.tdc[0][1] + s.tdc[1][1] + s.tdc[2][1] + s.tdc[3][1] < s.tdc[0][0] + s.tdc[1][0] + s.tdc[2][0] + s.tdc[3][0];
        }
        if (tr8) {
            // dct_luma8x8 [J] on one wave per 8x8 block, COEFF_COST8x8 thresholds as for 4x4
            int lev = 0, rv = 0, pv = 0;
            if (lu) {
                pv = s.pred[qy * 16 + qx];
                const int q8 = 16 + qp / 6;
                const int c = wave_fwd8x8(S_org[qy * 16 + qx] - pv, l8);
                int dq, cc;
                const unsigned long long nz = wave_quant8(c, l8, qp, q_round(d.qsel, q8), lev, dq, cc);
                rv = wave_inv8x8(dq, l8, pv, maxv);
                if (l8 == 0) { s.bcost[w8] = cc; s.bnz[w8] = nz != 0; }
            }
            __syncthreads();
            int sum_cnt = 0, keep8 = 0;
            for (int b8 = 0; b8 < 4; b8++) {
                int c8 = s.bcost[b8];
                if (c8 <= 4) c8 = 0;                                   // _LUMA_COEFF_COST_
                else {
                    keep8 |= 1 << b8;
                    if (s.bnz[b8]) { cbp |= 1 << b8; cbp_blk |= 0x33 << ((b8 >> 1) * 8 + (b8 & 1) * 2); }
                }
                sum_cnt += c8;
            }
            if (sum_cnt <= 5) { keep8 = 0; cbp = 0; cbp_blk = 0; }      // _LUMA_MB_COEFF_COST_
            if (lu) {
                const bool keep = (keep8 >> w8) & 1;
                s.lev[il_blk(w8, l8)][l8 >> 2] = keep ? (int16_t)lev : 0;
                s.rec[qy * 16 + qx] = (pel)(keep ? rv : pv);
            }
        } else {
        int lev = 0, rv = 0;
        if (lu) {
            const int c = lane_fwd4x4(S_org[py4 * 16 + px4] - p, l);
            int dq, cc;
            const int q_bits = 15 + qp / 6;
            unsigned nz = lane_quant(c, l, qp, q_round(d.qsel, q_bits), false, lev, dq, cc);
            rv = lane_inv4x4(dq, l, p, maxv);
            if (l == 0) { s.bcost[blk] = cc; s.bnz[blk] = nz != 0; }
        }
        __syncthreads();
        int sum_cnt = 0, keep8 = 0;
        for (int b8 = 0; b8 < 4; b8++) {
            int base = (b8 >> 1) * 8 + (b8 & 1) * 2;
            int c8 = s.bcost[base] + s.bcost[base + 1] + s.bcost[base + 4] + s.bcost[base + 5];
            int nz8 = s.bnz[base] | s.bnz[base + 1] | s.bnz[base + 4] | s.bnz[base + 5];
            if (c8 <= 4) c8 = 0;                                   // _LUMA_COEFF_COST_
            else {
                keep8 |= 1 << b8;
                if (nz8) cbp |= 1 << b8;
                for (int q = 0; q < 4; q++) {
                    int k = base + (q & 1) + (q >> 1) * 4;
                    if (s.bnz[k]) cbp_blk |= 1 << k;
                }
            }
            sum_cnt += c8;
        }
        if (sum_cnt <= 5) { keep8 = 0; cbp = 0; cbp_blk = 0; }      // _LUMA_MB_COEFF_COST_
        if (lu) {
            const int mb8 = ((blk >> 3) << 1) + ((blk & 3) >> 1);
            const bool keep = (keep8 >> mb8) & 1;
            s.lev[blk][l] = keep ? (int16_t)lev : 0;
            s.rec[py4 * 16 + px4] = (pel)(keep ? rv : p);
        }
        }
    }
    const bool t8flag = tr8 && (best_mode == JMH_I8MB || (cbp & 15));   // transform_size_8x8_flag
    PSTAMP(17);

    // ======== chroma: the rest of dct_chroma [J]
    if constexpr (!W2) chroma_a();
    __syncthreads();
    chroma_b();
    __syncthreads();
    chroma_c();
    __syncthreads();
    PSTAMP(18);
    int cr = 0;
    for (int uv = 0; uv < 2; uv++) {
        if (s.cdcnz[uv] & 1) cr = max(cr, 1);
        if (s.cdcnz[uv] & 2) cr = 2;
    }
    cbp |= cr << 4;

    // ======== outputs: jmh_mb_result, reconstruction, picture MV / ref / Intra4x4-mode arrays
    jmh_mb_result *res = d.res + mby * d.mbw + mbx;
    int mb_type = best_mode;
    if (slice_p && best_mode == 1 && cbp == 0 && s.fmv[0][0] == sc->skipx && s.fmv[0][1] == sc->skipy) mb_type = JMH_PSKIP;
    if (tid == 0) {
        res->mb_type = (int16_t)mb_type;
        res->cbp = (int16_t)cbp;
        res->cbp_blk = cbp_blk;
        for (int b = 0; b < 4; b++) {
            res->b8mode[b] = (int8_t)(mb_type == JMH_PSKIP ? 0 : b8mode[b]);
            res->ref_idx[b] = (int8_t)(is_intra ? -1 : 0);
        }
        res->i16mode = (int8_t)(best_mode == JMH_I16MB ? i16mode : 0);
        res->c_ipred_mode = (int8_t)c_mode;
        res->transform_8x8 = (int8_t)t8flag; res->pad0 = 0;
        res->min_cost = min_cost;
        res->reserved = 0;
    }
    if (lu) res->luma[blk][l] = s.lev[blk][l];
    if (tid < 16) {
        const int k = tid;
        const int ip = best_mode == JMH_I4MB ? sc->ipred[k]
                     : best_mode == JMH_I8MB ? (sc->i8modes >> (4 * (((k >> 3) << 1) + ((k & 3) >> 1)))) & 15 : 2;
        res->ipred[k] = (int8_t)ip;
        res->mv[k][0] = s.fmv[k][0]; res->mv[k][1] = s.fmv[k][1];
        res->luma_dc[k] = best_mode == JMH_I16MB ? s.dclev[k] : 0;
        const int a = ((pix_y >> 2) + (k >> 2)) * W4 + (pix_x >> 2) + (k & 3);
        d.mv[2 * a] = s.fmv[k][0]; d.mv[2 * a + 1] = s.fmv[k][1];
        d.refidx[a] = (int8_t)(is_intra ? -1 : 0);
        d.ipred[a] = (int8_t)ip;
    }
    if (tid < 8) { const int uv = tid >> 2, k = tid & 3; res->chroma_dc[uv][k] = s.cdc[uv][k]; }
    if (chv) {
        const int uv = ct >> 6, b = (ct >> 4) & 3, q = ct & 15;
        res->chroma_ac[uv][b][q] = s.cac[uv][b][q];
        const int k = ct & 63;
        (uv ? recV : recU)[((pix_y >> 1) + (k >> 3)) * Wc + (pix_x >> 1) + (k & 7)] = s.cfin[uv][k];
    }
    if (lu) recY[(pix_y + (tid >> 4)) * W + pix_x + (tid & 15)] = s.rec[tid];

    // ======== DeblockMb [J] / 8.7 into the reference picture (jmh_deblock.h)
    if (d.dbkY) deblock_mb<pel, NTH, true>(d, s.db, s.rec, s.cfin, s.fmv, is_intra, cbp_blk, t8flag, qpy, qpcy, mbx, mby, tid);
    PSTAMP(19);
}

// tick MB index m on threads tid = 0..NTH-1 of the workgroup (hwb: the hardware block, for the
// block profile; bt0 its start stamp)
template <int OCC, class pel, bool T8, int NTH = NT>
__device__ __forceinline__ void final_mb(const TickArgs &t, FinS<pel> &s, int m, int tid, int hwb, unsigned long long bt0) {
    const int e = tick_entry(t, m);
    const DevParams d = tick_params(t, e);
    const int mby = d.y_min + (m - t.pre[e]), mbx = d.diag - 2 * mby;
    // the 64-VGPR build samples the 6-tap's centre column by column: no spills (the unrolled form
    // spilled 56 B per lane and measured 0.9 % faster, profiles/r7b_c3_serialj_ab.txt)
    const pel *refY = spl<pel>(d.refY);
    const int W = d.W, H = d.H, maxv = sizeof(pel) == 1 ? 255 : d.maxv;
    auto mc = [=](int X, int Y) { return qpel_direct<pel, OCC == 8>(refY, W, H, X, Y, maxv); };
    final_core<OCC, pel, T8, NTH>(d, s, mbx, mby, tid, mc);
    if (t.bprof_fin && tid == 0) {
        t.bprof_fin[3 * hwb] = bt0;
        t.bprof_fin[3 * hwb + 1] = wall_clock64();
        t.bprof_fin[3 * hwb + 2] = 3;
    }
}

#endif
