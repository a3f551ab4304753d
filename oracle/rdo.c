/*
 * rdo.c — oracle restatement of JM lencod's encode_one_macroblock with RDOptimization = 1
 * (TEST INFRASTRUCTURE ONLY; see jm_oracle.h for the parity status).
 *
 * Restated JM 8.6 functions [J] (no file:line exists: /root/reference holds README.md:1-4):
 *   rdopt.c › encode_one_macroblock (the `input->rdopt` branches), RDCost_for_macroblocks,
 *             RDCost_for_8x8blocks, RDCost_for_4x4IntraBlocks, Mode_Decision_for_4x4IntraBlocks,
 *             SetCoeffAndReconstruction8x8, store_macroblock_parameters
 *   rdopt_coding_state.c › store_coding_state / reset_coding_state (a copy of the oracle's CABAC
 *             coder, cabac_enc.c: contexts, codILow, codIRange, outstanding bits)
 * with the entropy coder CABAC (SymbolMode 1), and with Transform8x8Mode 1 the JM FRExt additions
 * [J]: RDCost_for_8x8IntraBlocks (I8MB) and transform_size_8x8_flag per inter candidate (item 63).
 * Every non-normative choice is an item of docs/JM_SEMANTICS.md (53-60):
 *   - lambda_mode = fp.lambda_rd (0.85 * 2^((QP + QpBdOffsetY - 12) / 3), host libm), the searches'
 *     LAMBDA_FACTOR(sqrt(lambda_mode)) = fp.lambda_factor_rd; rdcost = (double)D + lambda * rate;
 *     candidates compared with strict '<' in JM's order;
 *   - D = SSD of the reconstruction (luma 16x16 + both 8x8 chroma) for the macroblock loop, of the
 *     8x8 / 4x4 luma block in the sub-decisions; rate = arienco_bits_written deltas of the oracle's
 *     own CABAC coder (cabac_enc.c) from the slice's coding state at the start of the macroblock
 *     (the P8x8 loop: the running state after the decided 8x8 blocks);
 *   - the motion searches are the RDO-off ones (items 3-10, 33-40) at the RDO lambda without the
 *     16x16 zero-vector biases (!input->rdopt) and with the RDO-off centre clamp kept (item 54).
 */
#include <stdlib.h>
#include "jmo_internal.h"

#define RD_HUGE 1e30

typedef struct {               /* a luma candidate of the macroblock loop                          */
    int mode;                  /* 0 (P_Skip), 1..3, JMH_P8x8, JMH_I16MB, JMH_I4MB, JMH_I8MB        */
    int t8;                    /* transform_size_8x8_flag of the candidate's luma                  */
    pel rec[256];
    int16_t luma[16][16], luma_dc[16];
    int cbp, cbp_blk;          /* luma cbp bits, 4x4 coded bits                                    */
    int16_t mv[16][2], mvd[16][2];
    int8_t ipm[16], imode[16]; /* I4 / I8: rem codes (-1 = predicted mode; I8 at each 8x8's top-left
                                  4x4), modes (I8: on the 8x8's four 4x4)                           */
    int i16mode, b8mode[4];
    int dist;                  /* luma SSD                                                         */
} lcand;
typedef struct {               /* a chroma candidate (an inter candidate's MC or an intra mode)    */
    pel rec[2][64];
    int16_t dc[2][4], ac[2][4][16];
    int cbpc, dist;
} ccand;

static int ssd(const pel *a, int as, const pel *b, int bs, int w, int h) {
    int d = 0;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int e = a[y * as + x] - b[y * bs + x];
            d += e * e;
        }
    return d;
}

/* LumaResidualCoding (RDO-off form): the prediction from the candidate's MVs, per 8x8
   LumaResidualCoding8x8 -- four dct_luma, or with L->t8 one dct_luma8x8 (levels in the CAVLC
   interleave of jmh_mb_result) -- with the _LUMA_COEFF_COST_ zeroing, then the MB-level one */
static void luma_inter(const mbs *s, int qp, int rnd, lcand *L, pel pred[256]) {
    const int maxv = s->c->maxv;
    for (int k = 0; k < 16; k++) jmo_luma_pred_4x4(s, k & 3, k >> 2, L->mv[k][0], L->mv[k][1], pred + 4 * (k >> 2) * 16 + 4 * (k & 3), 16);
    int sum = 0;
    L->cbp = L->cbp_blk = 0;
    memset(L->luma, 0, sizeof(L->luma));
    for (int b8 = 0; b8 < 4; b8++) {
        int cost = 0, cbp8 = 0, blk8 = 0;
        if (L->t8) {
            const int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
            int32_t r[64];
            int16_t lv[64];
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) r[8 * y + x] = s->org[(by + y) * 16 + bx + x] - pred[(by + y) * 16 + bx + x];
            if (jmo_dct_luma8x8(r, pred + by * 16 + bx, 16, qp, rnd, lv, &cost, L->rec + by * 16 + bx, 16, maxv)) {
                cbp8 = 1;
                blk8 = 0x33 << ((b8 >> 1) * 8 + (b8 & 1) * 2);
            }
            jmo_put_levels8(L->luma, b8, lv);
        } else
            for (int b4 = 0; b4 < 4; b4++) {
                int bx4 = 2 * (b8 & 1) + (b4 & 1), by4 = 2 * (b8 >> 1) + (b4 >> 1), k = by4 * 4 + bx4;
                int32_t r[16];
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++) r[4 * y + x] = s->org[(4 * by4 + y) * 16 + 4 * bx4 + x] - pred[(4 * by4 + y) * 16 + 4 * bx4 + x];
                if (jmo_dct_luma4x4(r, pred + 4 * by4 * 16 + 4 * bx4, 16, qp, rnd, L->luma[k], &cost, L->rec + 4 * by4 * 16 + 4 * bx4, 16,
                                    maxv)) { blk8 |= 1 << k; cbp8 = 1; }
            }
        if (cost <= LUMA_COEFF_COST) {
            cost = 0; cbp8 = 0; blk8 = 0;
            for (int b4 = 0; b4 < 4; b4++) {
                int bx4 = 2 * (b8 & 1) + (b4 & 1), by4 = 2 * (b8 >> 1) + (b4 >> 1);
                memset(L->luma[by4 * 4 + bx4], 0, 32);
                for (int y = 0; y < 4; y++) memcpy(L->rec + (4 * by4 + y) * 16 + 4 * bx4, pred + (4 * by4 + y) * 16 + 4 * bx4, 4 * sizeof(pel));
            }
        }
        if (cbp8) L->cbp |= 1 << b8;
        L->cbp_blk |= blk8;
        sum += cost;
    }
    if (sum <= LUMA_MB_COEFF_COST) {
        L->cbp = L->cbp_blk = 0;
        memset(L->luma, 0, sizeof(L->luma));
        memcpy(L->rec, pred, 256 * sizeof(pel));
    }
    L->dist = ssd(s->org, 16, L->rec, 16, 16, 16);
}

/* ChromaResidualCoding: prediction (intra mode cm, or MC with mv[]), dct_chroma unless skipped */
static void chroma_code(const mbs *s, int qpc, int rnd, const pel (*ipred)[4][64], int cm, const int16_t (*mv)[2], int skipped,
                        ccand *C) {
    C->cbpc = 0;
    C->dist = 0;
    for (int uv = 0; uv < 2; uv++) {
        pel pred[64];
        if (ipred) memcpy(pred, ipred[uv][cm], sizeof(pred));
        else jmo_chroma_pred_mb(s, uv, mv, pred);
        if (skipped) {
            memcpy(C->rec[uv], pred, sizeof(pred));
            memset(C->dc[uv], 0, sizeof(C->dc[uv]));
            memset(C->ac[uv], 0, sizeof(C->ac[uv]));
        } else {
            int32_t r[64];
            for (int k = 0; k < 64; k++) r[k] = s->orgc[uv][k] - pred[k];
            C->cbpc = jmo_dct_chroma(r, pred, qpc, rnd, C->cbpc, C->dc[uv], C->ac[uv], C->rec[uv], s->c->maxv);
        }
        C->dist += ssd(s->orgc[uv], 8, C->rec[uv], 8, 8, 8);
    }
}

static void fill_syn(jmo_cabsyn *r, const lcand *L, const ccand *C, int cm) {
    memset(r, 0, sizeof(*r));
    r->mb_type = L->mode;
    r->t8 = L->t8;
    r->cbp = L->cbp | C->cbpc << 4;
    r->i16mode = L->i16mode;
    r->cmode = cm;
    for (int b = 0; b < 4; b++) r->b8mode[b] = L->b8mode[b];
    for (int q = 0; q < 16; q++) { r->ipm[q] = L->ipm[q]; r->mvd[q][0] = L->mvd[q][0]; r->mvd[q][1] = L->mvd[q][1]; }
    r->luma = (const int16_t(*)[16])L->luma;
    r->luma_dc = L->luma_dc;
    r->cdc = (const int16_t(*)[4])C->dc;
    r->cac = (const int16_t(*)[4][16])C->ac;
}

/* the rate of one RD candidate: the bits the coder emits from `before` (hooked for the tests) */
static long rate_of(jmo_rate_event *ev, const jmo_cab *before, const jmo_cab *after) {
    ev->before = before;
    ev->after = after;
    ev->bits = jmo_cab_bits(after) - jmo_cab_bits(before);
    if (jmo_rate_hook) jmo_rate_hook(ev);
    return ev->bits;
}
/* ... with SymbolMode 0: the CAVLC bit count (cavlc_bits.c), tc_before the current MB's TotalCoeff
   the candidate was counted from */
static long rate_cav(jmo_rate_event *ev, const jmo_cavnb *cnb, const uint8_t *tc_before, long bits) {
    ev->cavlc = 1;
    ev->cnb = cnb;
    ev->tc_before = tc_before;
    ev->bits = bits;
    if (jmo_rate_hook) jmo_rate_hook(ev);
    return bits;
}

void jmo_encode_mb_rdo(jmo_ctx *c, int mbx, int mby) {
    mbs S;
    mbs *s = &S;
    memset(s, 0, sizeof(*s));
    s->c = c; s->mbx = mbx; s->mby = mby; s->pix_x = 16 * mbx; s->pix_y = 16 * mby;
    s->mb_addr = mby * c->mbw + mbx;
    s->lf = c->fp.lambda_factor_rd;
    s->lambda = c->fp.lambda_mode;
    s->rdo = 1;
    s->slice_p = c->fp.slice_type == JMH_P_SLICE;
    const double lam = c->fp.lambda_rd;
    const int qpy = c->fp.qp, qp = qpy + c->qpbd, maxv = c->maxv, W = c->W, W4 = W >> 2;
    const int jm10 = c->cfg.jm_version >= 10;
    const int rnd = jm10 ? JMO_RND_OFF(c->cfg.quant_offset[s->slice_p]) : !s->slice_p;
    const int i16_rnd = jm10 ? rnd : JMO_RND_I;
    const int qpc = jmo_qpc(qpy + c->fp.chroma_qp_offset, c->qpbd) + c->qpbd;
    for (int y = 0; y < 16; y++) memcpy(s->org + 16 * y, c->orgY + (s->pix_y + y) * W + s->pix_x, 16 * sizeof(pel));
    for (int y = 0; y < 8; y++) {
        memcpy(s->orgc[0] + 8 * y, c->orgU + ((s->pix_y >> 1) + y) * c->Wc + (s->pix_x >> 1), 8 * sizeof(pel));
        memcpy(s->orgc[1] + 8 * y, c->orgV + ((s->pix_y >> 1) + y) * c->Wc + (s->pix_x >> 1), 8 * sizeof(pel));
    }
    /* the slice's coding state: initialised at its first macroblock (9.3.1) */
    const int a = s->mb_addr, nmb = c->mbw * c->mbh, k = c->cfg.slice_mbs > 0 ? c->cfg.slice_mbs : nmb;
    const int cavlc = c->cfg.symbol_mode == 0;              /* SymbolMode 0: CAVLC rates (item 64) */
    if (a % k == 0) {
        if (cavlc) c->cav_run = 0;
        else jmo_cab_start(&c->cab, !s->slice_p, qpy);
    }
    jmo_cabnb nb;
    memset(&nb, 0, sizeof(nb));
    nb.A = mbx > 0 && jmo_same_slice(c, a, a - 1) ? &c->cabi[a - 1] : NULL;
    nb.B = mby > 0 && jmo_same_slice(c, a, a - c->mbw) ? &c->cabi[a - c->mbw] : NULL;
    for (int r = 0; r < 4; r++)
        for (int comp = 0; comp < 2; comp++) {
            if (nb.A) nb.mvdA[r][comp] = c->cab_mvd[2 * ((4 * mby + r) * W4 + 4 * mbx - 1) + comp];
            if (nb.B) nb.mvdB[r][comp] = c->cab_mvd[2 * ((4 * mby - 1) * W4 + 4 * mbx + r) + comp];
        }
    jmo_cab e;
    jmo_rate_event ev;
    jmo_cavnb cnb = {nb.A ? c->cav_tc + (size_t)(a - 1) * 24 : NULL, nb.B ? c->cav_tc + (size_t)(a - c->mbw) * 24 : NULL};
#define RATE_BEGIN(kind_) (e = c->cab, memset(&ev, 0, sizeof(ev)), ev.kind = (kind_), ev.slice_p = s->slice_p, ev.nb = &nb)

    const int *isr = c->cfg.inter_search;
    int valid[9] = {0};
    for (int m = 1; m <= 7; m++) valid[m] = s->slice_p && isr[m];
    valid[8] = valid[4] || valid[5] || valid[6] || valid[7];

    /* candidates (one MB at a time): 0 skip, 1..3, 4 P8x8, 5 I16, 6 I4, 7 I8; Transform8x8Mode:
       8..10 the 16x16 / 16x8 / 8x16 and 11 the P8x8 (all sub-modes 8x8) with the 8x8 transform */
    enum { NC = 12 };
    static lcand Lc[NC];
    int have[NC] = {0};
    const int t8m = c->cfg.transform_8x8_mode;
    pel pred[256];
    if (s->slice_p) {
        /* ===== motion estimation for 16x16, 16x8, 8x16 (PartitionMotionSearch) ===== */
        for (int mode = 1; mode < 4; mode++)
            if (valid[mode])
                for (int block = 0; block < (mode == 1 ? 1 : 2); block++) jmo_partition_motion_search(s, mode, block);
        /* ===== P8x8: per 8x8 block the sub-modes 4..7 by RDCost_for_8x8blocks ===== */
        if (valid[8]) {
            lcand *P = &Lc[4];
            memset(P, 0, sizeof(*P));
            P->mode = JMH_P8x8;
            static jmo_cab st8, stb, stc;
            st8 = c->cab;
            jmo_cabcur cur, curb;
            memset(&cur, 0, sizeof(cur));
            curb = cur;
            uint8_t ctc[24] = {0}, ctcb[24] = {0};        /* CAVLC: the decided blocks' TotalCoeff */
            pel pred8[256], rec8[256];
            int cnt_nonz = 0;
            for (int block = 0; block < 4; block++) {
                const int ox = 8 * (block & 1), oy = 8 * (block >> 1);
                double best = RD_HUGE;
                int bm = 0, bcost = 0, bcbp = 0, bblk = 0;
                int16_t blev[4][16];
                pel bpred[64], brec[64];
                for (int mode = 4; mode <= 7; mode++) {
                    if (!valid[mode]) continue;
                    jmo_partition_motion_search(s, mode, block);
                    /* LumaResidualCoding8x8 */
                    pel p8[64], r8[64];
                    int16_t lev[4][16];
                    int cost = 0, cbpbit = 0, blk = 0;
                    for (int b4 = 0; b4 < 4; b4++) {
                        int bx4 = 2 * (block & 1) + (b4 & 1), by4 = 2 * (block >> 1) + (b4 >> 1), kk = by4 * 4 + bx4;
                        int px = 4 * (b4 & 1), py = 4 * (b4 >> 1);
                        jmo_luma_pred_4x4(s, bx4, by4, s->all_mv[mode][kk][0], s->all_mv[mode][kk][1], p8 + py * 8 + px, 8);
                        int32_t r[16];
                        for (int y = 0; y < 4; y++)
                            for (int x = 0; x < 4; x++) r[4 * y + x] = s->org[(oy + py + y) * 16 + ox + px + x] - p8[(py + y) * 8 + px + x];
                        if (jmo_dct_luma4x4(r, p8 + py * 8 + px, 8, qp, rnd, lev[b4], &cost, r8 + py * 8 + px, 8, maxv)) {
                            cbpbit = 1; blk |= 1 << kk;
                        }
                    }
                    if (cost <= LUMA_COEFF_COST) {
                        cost = 0; cbpbit = 0; blk = 0;
                        memset(lev, 0, sizeof(lev));
                        memcpy(r8, p8, sizeof(r8));
                    }
                    int D = ssd(s->org + oy * 16 + ox, 16, r8, 8, 8, 8);
                    /* rate: sub_mb_type, mvds, cbp bit, luma (RDCost_for_8x8blocks) */
                    int16_t mvd[4][2];
                    for (int b4 = 0; b4 < 4; b4++) {
                        int kk = (2 * (block >> 1) + (b4 >> 1)) * 4 + 2 * (block & 1) + (b4 & 1);
                        mvd[b4][0] = (int16_t)(s->all_mv[mode][kk][0] - s->pmv[mode][kk][0]);
                        mvd[b4][1] = (int16_t)(s->all_mv[mode][kk][1] - s->pmv[mode][kk][1]);
                    }
                    jmo_rate_event eb;
                    memset(&eb, 0, sizeof(eb));
                    eb.kind = JMO_RATE_B8; eb.slice_p = 1; eb.nb = &nb; eb.cur_before = &cur;
                    eb.b8 = block; eb.sm = mode; eb.coded = cost > 0;
                    eb.mvd4 = (const int16_t(*)[2])mvd; eb.lev4 = (const int16_t(*)[16])lev;
                    jmo_cabcur cc = cur;
                    uint8_t tcc[24];
                    long bits;
                    if (cavlc) {
                        memcpy(tcc, ctc, 24);
                        bits = rate_cav(&eb, &cnb, ctc, jmo_cavlc_b8_bits(&cnb, tcc, block, mode, (const int16_t(*)[2])mvd, cost > 0,
                                                                        (const int16_t(*)[16])lev));
                    } else {
                        stc = st8;
                        jmo_cab_b8(&stc, &nb, &cc, block, mode, (const int16_t(*)[2])mvd, cost > 0, (const int16_t(*)[16])lev);
                        bits = rate_of(&eb, &st8, &stc);
                    }
                    double rd = (double)D + lam * (double)bits;
                    if (rd < best) {
                        best = rd; bm = mode; bcost = cost; bcbp = cbpbit; bblk = blk;
                        memcpy(blev, lev, sizeof(blev)); memcpy(bpred, p8, sizeof(bpred)); memcpy(brec, r8, sizeof(brec));
                        if (cavlc) memcpy(ctcb, tcc, 24);
                        else { stb = stc; curb = cc; }
                    }
                }
                /* the block's decision: coding state, SetRefAndMotionVectors, stored coefficients */
                if (cavlc) memcpy(ctc, ctcb, 24);
                else { st8 = stb; cur = curb; }
                P->b8mode[block] = bm;
                jmo_write_enc_mv(s, 2 * (block & 1), 2 * (block >> 1), 2, 2, s->all_mv[bm]);
                for (int b4 = 0; b4 < 4; b4++) {
                    int bx4 = 2 * (block & 1) + (b4 & 1), by4 = 2 * (block >> 1) + (b4 >> 1), kk = by4 * 4 + bx4;
                    memcpy(P->luma[kk], blev[b4], 32);
                    P->mv[kk][0] = s->all_mv[bm][kk][0]; P->mv[kk][1] = s->all_mv[bm][kk][1];
                    P->mvd[kk][0] = (int16_t)(s->all_mv[bm][kk][0] - s->pmv[bm][kk][0]);
                    P->mvd[kk][1] = (int16_t)(s->all_mv[bm][kk][1] - s->pmv[bm][kk][1]);
                }
                for (int y = 0; y < 8; y++) {
                    memcpy(pred8 + (oy + y) * 16 + ox, bpred + 8 * y, 8 * sizeof(pel));
                    memcpy(rec8 + (oy + y) * 16 + ox, brec + 8 * y, 8 * sizeof(pel));
                }
                if (bcost) { P->cbp |= bcbp << block; P->cbp_blk |= bblk; cnt_nonz += bcost; }
            }
            /* SetCoeffAndReconstruction8x8 */
            if (cnt_nonz <= LUMA_MB_COEFF_COST) {
                P->cbp = P->cbp_blk = 0;
                memset(P->luma, 0, sizeof(P->luma));
                memcpy(P->rec, pred8, sizeof(pred8));
            } else memcpy(P->rec, rec8, sizeof(rec8));
            P->dist = ssd(s->org, 16, P->rec, 16, 16, 16);
            have[4] = 1;
        }
        jmo_find_skip_mv(s);
        memcpy(c->mem_mv, s->all_mv, sizeof(c->mem_mv));   /* EPZS spatial memory of the next MB */
        /* the inter candidates of the macroblock loop */
        lcand *K = &Lc[0];
        memset(K, 0, sizeof(*K));
        K->mode = 0;
        for (int q = 0; q < 16; q++) { K->mv[q][0] = (int16_t)s->skip_mv[0]; K->mv[q][1] = (int16_t)s->skip_mv[1]; }
        for (int q = 0; q < 16; q++) jmo_luma_pred_4x4(s, q & 3, q >> 2, K->mv[q][0], K->mv[q][1], K->rec + 4 * (q >> 2) * 16 + 4 * (q & 3), 16);
        K->dist = ssd(s->org, 16, K->rec, 16, 16, 16);
        have[0] = 1;
        for (int mode = 1; mode < 4; mode++) {
            if (!valid[mode]) continue;
            lcand *L = &Lc[mode];
            memset(L, 0, sizeof(*L));
            L->mode = mode;
            for (int q = 0; q < 16; q++) {
                L->mv[q][0] = s->all_mv[mode][q][0]; L->mv[q][1] = s->all_mv[mode][q][1];
                L->mvd[q][0] = (int16_t)(s->all_mv[mode][q][0] - s->pmv[mode][q][0]);
                L->mvd[q][1] = (int16_t)(s->all_mv[mode][q][1] - s->pmv[mode][q][1]);
                L->b8mode[q & 3] = mode;
            }
            luma_inter(s, qp, rnd, L, pred);
            have[mode] = 1;
        }
        /* Transform8x8Mode: the same motion with transform_size_8x8_flag 1 (item 63) */
        for (int mode = 1; t8m && mode <= 4; mode++) {
            if (!have[mode] || (mode == 4 && !(Lc[4].b8mode[0] == 4 && Lc[4].b8mode[1] == 4 && Lc[4].b8mode[2] == 4 &&
                                               Lc[4].b8mode[3] == 4))) continue;
            lcand *L = &Lc[mode + 7];
            *L = Lc[mode];
            L->t8 = 1;
            luma_inter(s, qp, rnd, L, pred);
            have[mode + 7] = 1;
        }
    }

    /* ===== Intra16x16: the find_sad_16x16 mode, dct_luma_16x16 ===== */
    {
        lcand *L = &Lc[5];
        memset(L, 0, sizeof(*L));
        L->mode = JMH_I16MB;
        pel ip[4][256];
        int av[4], m = 2;
        jmo_intra16_pred(s, ip, av);
        jmo_find_sad_16x16(s, ip, av, &m);
        int32_t r[256];
        for (int q = 0; q < 256; q++) r[q] = s->org[q] - ip[m][q];
        L->cbp = jmo_dct_luma_16x16(r, ip[m], qp, i16_rnd, L->luma_dc, L->luma, &L->cbp_blk, L->rec, maxv);
        L->i16mode = m;
        L->dist = ssd(s->org, 16, L->rec, 16, 16, 16);
        have[5] = 1;
    }
    /* ===== Intra4x4: Mode_Decision_for_4x4IntraBlocks by RDCost_for_4x4IntraBlocks ===== */
    {
        lcand *L = &Lc[6];
        memset(L, 0, sizeof(*L));
        L->mode = JMH_I4MB;
        uint8_t i4tc[24] = {0};                         /* CAVLC: the decided blocks' TotalCoeff */
        for (int b8 = 0; b8 < 4; b8++)
            for (int b4 = 0; b4 < 4; b4++) {
                int bx = 8 * (b8 & 1) + 4 * (b4 & 1), by = 8 * (b8 >> 1) + 4 * (b4 >> 1), q = (by >> 2) * 4 + (bx >> 2);
                int ia = 0, ib = 0;
                int av_l = jmo_nb4(s, bx - 1, by, &ia), av_u = jmo_nb4(s, bx, by - 1, &ib);
                int up = av_u ? c->ipred[ib] : -1, left = av_l ? c->ipred[ia] : -1;
                int mpm = (up < 0 || left < 0) ? 2 : imin(up, left);
                pel ip[9][16];
                int av[9];
                jmo_intra4x4_pred(s, bx, by, ip, av);
                double best = RD_HUGE;
                int bmode = 2, bnz = 0;
                int16_t blev[16];
                pel brec[16];
                uint8_t btc[24];
                for (int m = 0; m < 9; m++) {
                    if (!av[m]) continue;
                    int32_t r[16];
                    for (int y = 0; y < 4; y++)
                        for (int x = 0; x < 4; x++) r[4 * y + x] = s->org[(by + y) * 16 + bx + x] - ip[m][4 * y + x];
                    int16_t lev[16];
                    pel rec4[16];
                    int dummy = 0;
                    int nz = jmo_dct_luma4x4(r, ip[m], 4, qp, rnd, lev, &dummy, rec4, 4, maxv);
                    int D = ssd(s->org + by * 16 + bx, 16, rec4, 4, 4, 4);
                    RATE_BEGIN(JMO_RATE_I4);
                    ev.x4 = bx >> 2; ev.y4 = by >> 2; ev.code = m == mpm ? -1 : m < mpm ? m : m - 1; ev.lev = lev;
                    uint8_t tcc[24];
                    long bits;
                    if (cavlc) {
                        memcpy(tcc, i4tc, 24);
                        bits = rate_cav(&ev, &cnb, i4tc, jmo_cavlc_i4_bits(&cnb, tcc, ev.x4, ev.y4, ev.code, lev));
                    } else {
                        jmo_cab_i4(&e, &nb, ev.x4, ev.y4, ev.code, lev);
                        bits = rate_of(&ev, &c->cab, &e);
                    }
                    double rd = (double)D + lam * (double)bits;
                    if (rd < best) {
                        best = rd; bmode = m; bnz = nz; memcpy(blev, lev, sizeof(blev)); memcpy(brec, rec4, sizeof(brec));
                        if (cavlc) memcpy(btc, tcc, 24);
                    }
                }
                if (cavlc) memcpy(i4tc, btc, 24);
                c->ipred[((s->pix_y + by) >> 2) * W4 + ((s->pix_x + bx) >> 2)] = (int8_t)bmode;
                for (int y = 0; y < 4; y++) memcpy(c->recY + (s->pix_y + by + y) * W + s->pix_x + bx, brec + 4 * y, 4 * sizeof(pel));
                memcpy(L->luma[q], blev, sizeof(blev));
                L->imode[q] = (int8_t)bmode;
                L->ipm[q] = (int8_t)(bmode == mpm ? -1 : bmode < mpm ? bmode : bmode - 1);
                if (bnz) { L->cbp |= 1 << b8; L->cbp_blk |= 1 << q; }
            }
        for (int y = 0; y < 16; y++) memcpy(L->rec + 16 * y, c->recY + (s->pix_y + y) * W + s->pix_x, 16 * sizeof(pel));
        L->dist = ssd(s->org, 16, L->rec, 16, 16, 16);
        have[6] = 1;
    }
    /* ===== Intra8x8 (Transform8x8Mode): Mode_Decision_for_8x8IntraBlocks by RDCost_for_8x8IntraBlocks
       per 8x8 block -- 8x8 TQ, D = SSD of the block, R = the pred-mode syntax + the 8x8 residual
       from the state at the macroblock start; strict '<' over modes 0..8; the winner reconstructs
       before the next block (item 63) ===== */
    if (t8m) {
        lcand *L = &Lc[7];
        memset(L, 0, sizeof(*L));
        L->mode = JMH_I8MB;
        L->t8 = 1;
        int modes[4] = {2, 2, 2, 2};
        uint8_t i8tc[24] = {0};                         /* CAVLC: the decided blocks' TotalCoeff */
        for (int b8 = 0; b8 < 4; b8++) {
            const int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
            int32_t nbs[25];
            const int avb = jmo_i8_neighbours(s, L->rec, b8, nbs);
            pel ip[9][64];
            const int ok = jmo_intra8x8_pred_px(nbs, avb, ip, (maxv + 1) >> 1);
            const int mpm = jmo_i8_mpm(s, b8, modes);
            double best = RD_HUGE;
            int bmode = 2, bnz = 0;
            int16_t blev[64];
            pel brec[64];
            uint8_t btc[24];
            for (int m = 0; m < 9; m++) {
                if (!((ok >> m) & 1)) continue;
                int32_t r[64];
                for (int y = 0; y < 8; y++)
                    for (int x = 0; x < 8; x++) r[8 * y + x] = s->org[(by + y) * 16 + bx + x] - ip[m][8 * y + x];
                int16_t lev[64];
                pel rec8[64];
                int dummy = 0;
                const int nz = jmo_dct_luma8x8(r, ip[m], 8, qp, rnd, lev, &dummy, rec8, 8, maxv);
                const int D = ssd(s->org + by * 16 + bx, 16, rec8, 8, 8, 8);
                RATE_BEGIN(JMO_RATE_I8);
                ev.code = m == mpm ? -1 : m < mpm ? m : m - 1;
                ev.lev = lev;
                ev.b8i = b8;
                uint8_t tcc[24];
                long bits;
                if (cavlc) {
                    memcpy(tcc, i8tc, 24);
                    bits = rate_cav(&ev, &cnb, i8tc, jmo_cavlc_i8_bits(&cnb, tcc, b8, ev.code, lev));
                } else {
                    jmo_cab_i8(&e, ev.code, lev);
                    bits = rate_of(&ev, &c->cab, &e);
                }
                double rd = (double)D + lam * (double)bits;
                if (rd < best) {
                    best = rd; bmode = m; bnz = nz; memcpy(blev, lev, sizeof(blev)); memcpy(brec, rec8, sizeof(brec));
                    if (cavlc) memcpy(btc, tcc, 24);
                }
            }
            if (cavlc) memcpy(i8tc, btc, 24);
            modes[b8] = bmode;
            for (int y = 0; y < 8; y++) memcpy(L->rec + (by + y) * 16 + bx, brec + 8 * y, 8 * sizeof(pel));
            jmo_put_levels8(L->luma, b8, blev);
            L->ipm[(b8 >> 1) * 8 + (b8 & 1) * 2] = (int8_t)(bmode == mpm ? -1 : bmode < mpm ? bmode : bmode - 1);
            for (int q = 0; q < 16; q++)
                if (((q >> 3) << 1) + ((q & 3) >> 1) == b8) L->imode[q] = (int8_t)bmode;
            if (bnz) { L->cbp |= 1 << b8; L->cbp_blk |= 0x33 << ((b8 >> 1) * 8 + (b8 & 1) * 2); }
        }
        L->dist = ssd(s->org, 16, L->rec, 16, 16, 16);
        have[7] = 1;
    }

    /* ===== chroma candidates: each inter candidate's MC, the intra modes ===== */
    static ccand Cc[5], Ci[4];
    pel cip[2][4][64];
    int cav[4];
    jmo_intra_chroma_pred(s, 0, cip[0], cav);
    jmo_intra_chroma_pred(s, 1, cip[1], cav);
    for (int i = 0; i < 5; i++)
        if (have[i]) chroma_code(s, qpc, rnd, NULL, 0, (const int16_t(*)[2])Lc[i].mv, i == 0, &Cc[i]);
    for (int cm = 0; cm < 4; cm++)
        if (cav[cm]) chroma_code(s, qpc, rnd, (const pel(*)[4][64])cip, cm, NULL, 0, &Ci[cm]);

    /* ===== RDCost_for_macroblocks over c_ipred_mode (outer) and the modes (inner), JM order:
       0, 1, 2, 3, P8x8 (each with the 4x4 then the 8x8 transform), I16MB, I4MB, I8MB ===== */
    static const int order[NC] = {0, 1, 8, 2, 9, 3, 10, 4, 11, 5, 6, 7};
#define CBASE(i) ((i) >= 8 ? (i) - 7 : (i))                  /* an inter candidate's chroma */
    double min_rd = RD_HUGE;
    int bi = -1, bcm = 0, brate = 0;
    for (int cm = 0; cm < 4; cm++) {
        if (!cav[cm]) continue;
        for (int oi = 0; oi < NC; oi++) {
            int i = order[oi], intra = i >= 5 && i <= 7;
            if (!have[i] || (cm != 0 && !intra)) continue;
            const ccand *C = intra ? &Ci[cm] : &Cc[CBASE(i)];
            jmo_cabsyn r;
            long bits;
            if (i == 0) {
                RATE_BEGIN(JMO_RATE_SKIP);
                if (cavlc) {   /* the run is written with the next coded MB, or here at the picture's last MB */
                    ev.skip_run = c->cav_run;
                    ev.last_mb = a == nmb - 1;
                    bits = rate_cav(&ev, &cnb, NULL, jmo_cavlc_skip_bits(c->cav_run, a == nmb - 1));
                }
                else {
                    jmo_cab_skip(&e, &nb);
                    bits = rate_of(&ev, &c->cab, &e);
                }
            } else {
                RATE_BEGIN(JMO_RATE_MB);
                fill_syn(&r, &Lc[i], C, intra ? cm : 0);
                ev.syn = &r;
                ev.t8mode = t8m;
                if (cavlc) {
                    ev.skip_run = c->cav_run;
                    bits = rate_cav(&ev, &cnb, NULL, jmo_cavlc_mb_bits(&cnb, &r, s->slice_p, t8m, c->cav_run, NULL));
                } else {
                    jmo_cab_mb(&e, &nb, &r, s->slice_p, t8m, NULL, NULL);
                    bits = rate_of(&ev, &c->cab, &e);
                }
            }
            double rd = (double)(Lc[i].dist + C->dist) + lam * (double)bits;
            if (rd < min_rd) { min_rd = rd; bi = i; bcm = intra ? cm : 0; brate = (int)bits; }
        }
    }

    /* ===== the chosen macroblock: results, reconstruction, picture arrays, coding state ===== */
    const lcand *L = &Lc[bi];
    const int is_intra = bi >= 5 && bi <= 7;
    const ccand *C = is_intra ? &Ci[bcm] : &Cc[CBASE(bi)];
#undef CBASE
    jmh_mb_result *res = &c->res[a];
    memset(res, 0, sizeof(*res));
    int mb_type = L->mode == 0 ? JMH_PSKIP : L->mode;
    res->mb_type = (int16_t)mb_type;
    res->cbp = (int16_t)(L->cbp | C->cbpc << 4);
    res->cbp_blk = L->cbp_blk;
    for (int b = 0; b < 4; b++) {
        res->b8mode[b] = (int8_t)(mb_type == JMH_PSKIP ? 0 : mb_type == JMH_P8x8 ? L->b8mode[b] : mb_type == JMH_I4MB ? JMH_IBLOCK
                                                   : mb_type == JMH_I16MB ? 0 : mb_type);
        res->ref_idx[b] = (int8_t)(is_intra ? -1 : 0);
    }
    res->transform_8x8 = (int8_t)(L->t8 && (mb_type == JMH_I8MB || (L->cbp & 15)));
    res->i16mode = (int8_t)(mb_type == JMH_I16MB ? L->i16mode : 0);
    res->c_ipred_mode = (int8_t)(is_intra ? bcm : 0);
    res->min_cost = brate;                                /* the chosen candidate's rate (bits) */
    memcpy(res->luma, L->luma, sizeof(res->luma));
    memcpy(res->luma_dc, L->luma_dc, sizeof(res->luma_dc));
    memcpy(res->chroma_dc, C->dc, sizeof(res->chroma_dc));
    memcpy(res->chroma_ac, C->ac, sizeof(res->chroma_ac));
    for (int q = 0; q < 16; q++) {
        res->mv[q][0] = is_intra ? 0 : L->mv[q][0];
        res->mv[q][1] = is_intra ? 0 : L->mv[q][1];
        res->ipred[q] = (int8_t)(mb_type == JMH_I4MB || mb_type == JMH_I8MB ? L->imode[q] : 2);
        int pa = ((s->pix_y >> 2) + (q >> 2)) * W4 + (s->pix_x >> 2) + (q & 3);
        c->mv[2 * pa] = res->mv[q][0];
        c->mv[2 * pa + 1] = res->mv[q][1];
        c->refidx[pa] = (int8_t)(is_intra ? -1 : 0);
        c->ipred[pa] = (int8_t)(!is_intra && c->cfg.constrained_intra_pred ? -1 : res->ipred[q]);   /* (8.3.1.1, as encode.c) */
    }
    c->mbintra[a] = (int8_t)is_intra;
    jmo_store_rec_luma(c, s, L->rec);
    for (int uv = 0; uv < 2; uv++) {
        pel *R = uv ? c->recV : c->recU;
        for (int y = 0; y < 8; y++) memcpy(R + ((s->pix_y >> 1) + y) * c->Wc + (s->pix_x >> 1), C->rec[uv] + 8 * y, 8 * sizeof(pel));
    }
    /* write_one_macroblock: the coding state advances by the chosen macroblock (what it leaves for
       its neighbours' contexts: jmo_cabmbi, the mvds of its 4x4 blocks), then the end_of_slice_flag
       (0) unless the slice ends here */
    int16_t mvd[16][2];
    memset(mvd, 0, sizeof(mvd));
    if (cavlc) {                                          /* CAVLC: the skip run, the TotalCoeff */
        uint8_t *tco = c->cav_tc + (size_t)a * 24;
        if (bi == 0) { c->cav_run++; memset(tco, 0, 24); }
        else {
            jmo_cabsyn r;
            fill_syn(&r, L, C, is_intra ? bcm : 0);
            jmo_cavlc_mb_bits(&cnb, &r, s->slice_p, t8m, c->cav_run, tco);
            c->cav_run = 0;
        }
    } else if (bi == 0) {
        jmo_cab_skip(&c->cab, &nb);
        memset(&c->cabi[a], 0, sizeof(c->cabi[a]));
        c->cabi[a].skip = 1;
    } else {
        jmo_cabsyn r;
        fill_syn(&r, L, C, is_intra ? bcm : 0);
        jmo_cab_mb(&c->cab, &nb, &r, s->slice_p, t8m, &c->cabi[a], mvd);
    }
    for (int q = 0; q < 16; q++) {
        const int pa = ((s->pix_y >> 2) + (q >> 2)) * W4 + (s->pix_x >> 2) + (q & 3);
        c->cab_mvd[2 * pa] = mvd[q][0];
        c->cab_mvd[2 * pa + 1] = mvd[q][1];
    }
    if (!cavlc && (a + 1) % k != 0 && a + 1 < nmb) jmo_cab_terminate(&c->cab, 0);
#undef RATE_BEGIN
}
