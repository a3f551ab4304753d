/*
 * cabac_enc.c — the oracle's own CABAC coder: the rate of RDOptimization 1 (TEST INFRASTRUCTURE ONLY;
 * see jm_oracle.h for the parity status).
 *
 * JM's RD loop [J] codes every candidate with its real arithmetic coder between store_coding_state
 * and reset_coding_state (rdopt_coding_state.c) and takes
 *     rate = arienco_bits_written(after) - arienco_bits_written(before)          (biariencode.c)
 * with arienco_bits_written = 8 * bytes + 8 - Ebits_to_go + Ebits_to_follow (the first bit of a
 * slice is shifted out of a 9-bit first byte: the count starts at -1).  This file restates that
 * coder from ITU-T H.264 9.3.4 as written — codILow, codIRange, PutBit with firstBitFlag and
 * bitsOutstanding, EncodeDecision / EncodeBypass / EncodeTerminate with RenormE — and counts the
 * bits the way JM counts them.  Binarisations (9.3.2) and ctxIdxInc derivations (9.3.3.1) follow the
 * spec clauses one syntax element at a time over spec ctxIdx numbering, with the context tables of
 * the independent decoder (decoder.c: Tables 9-12..9-33, 9-43, 9-44, proven by its closed loop).
 *
 * It shares no code with the product: csrc/jmh_cabac_rate.h counts renormalisation steps over a
 * dense context space without codILow, host/cabac.c writes the bitstream.  tests/test_rate_xcheck.py
 * compares the product's rate engine with this coder on every candidate of every macroblock (the
 * hook below), including the losing ones.
 */
#include <stdlib.h>
#include "jmo_internal.h"

void (*jmo_rate_hook)(const jmo_rate_event *ev) = NULL;

/* ---- the arithmetic coder (9.3.4.2 .. 9.3.4.5) ------------------------------------------ */
void jmo_cab_start(jmo_cab *e, int slice_i, int qp) {       /* 9.3.1.1 + 9.3.4.1 */
    jmo_cabac_init_models(slice_i, qp, e->st, e->mps);
    e->low = 0;
    e->range = 510;
    e->first = 1;
    e->outstanding = 0;
    e->put = 0;
}
long jmo_cab_bits(const jmo_cab *e) { return e->put + e->outstanding - 1; }

static void put_bit(jmo_cab *e, int b) {                   /* PutBit (Figure 9-8) */
    (void)b;                                                /* only the count matters here */
    if (e->first) e->first = 0;                             /* not written; JM counts it in its 9-bit first byte */
    e->put += 1 + e->outstanding;
    e->outstanding = 0;
}
static void renorm(jmo_cab *e) {                           /* RenormE (Figure 9-7) */
    while (e->range < 256) {
        if (e->low < 256) put_bit(e, 0);
        else if (e->low >= 512) { e->low -= 512; put_bit(e, 1); }
        else { e->low -= 256; e->outstanding++; }
        e->range <<= 1;
        e->low <<= 1;
    }
}
void jmo_cab_decision(jmo_cab *e, int ctx, int bin) {     /* EncodeDecision (Figure 9-6) */
    const int s = e->st[ctx];
    const uint32_t lps = jmo_lps_range[s][(e->range >> 6) & 3];
    e->range -= lps;
    if (bin != e->mps[ctx]) {
        e->low += e->range;
        e->range = lps;
        if (s == 0) e->mps[ctx] = (uint8_t)(1 - e->mps[ctx]);
        e->st[ctx] = jmo_lps_next[s];
    } else if (s < 62) e->st[ctx] = (uint8_t)(s + 1);      /* transIdxMPS (Table 9-45) */
    renorm(e);
}
void jmo_cab_bypass(jmo_cab *e, int bin) {                 /* EncodeBypass (Figure 9-9) */
    e->low <<= 1;
    if (bin) e->low += e->range;
    if (e->low >= 1024) { put_bit(e, 1); e->low -= 1024; }
    else if (e->low < 512) put_bit(e, 0);
    else { e->low -= 512; e->outstanding++; }
}
void jmo_cab_terminate(jmo_cab *e, int bin) {              /* EncodeTerminate (Figure 9-10) */
    e->range -= 2;
    if (bin) {                                              /* EncodeFlush: the count only */
        e->low += e->range;
        e->range = 2;
        renorm(e);
        put_bit(e, (e->low >> 9) & 1);
        e->put += 2;                                        /* WriteBits(((codILow >> 7) & 3) | 1, 2) */
    } else renorm(e);
}

/* UEGk suffix, k-th order Exp-Golomb in bypass bins (9.3.2.3) */
static void eg_bypass(jmo_cab *e, unsigned v, int k) {
    for (;;) {
        if (v >= (1u << k)) { jmo_cab_bypass(e, 1); v -= 1u << k; k++; }
        else {
            jmo_cab_bypass(e, 0);
            while (k--) jmo_cab_bypass(e, (v >> k) & 1);
            return;
        }
    }
}

/* ---- ctxIdxInc of the neighbour-dependent elements (9.3.3.1.1) --------------------------- */
static int avail_coded(const jmo_cabmbi *n) { return n && !n->skip; }

/* condTermFlagN of coded_block_flag for a luma 4x4 block (x4, y4) of neighbour n (9.3.3.1.1.9):
   unavailable -> the current macroblock is intra; P_Skip or its 8x8 block without coded luma -> 0;
   otherwise the block's coded_block_flag (an 8x8-transform block's flag is inferred 1 and stored
   on its four 4x4 positions) */
static int cbf_term_luma(const jmo_cabmbi *n, int cur_intra, int x4, int y4) {
    if (!n) return cur_intra;
    if (n->skip) return 0;
    if (!((n->cbp >> ((y4 >> 1) * 2 + (x4 >> 1))) & 1)) return 0;
    return (n->cbf4 >> (y4 * 4 + x4)) & 1;
}
static int cbf_term_cdc(const jmo_cabmbi *n, int cur_intra, int uv) {
    if (!n) return cur_intra;
    if (n->skip || (n->cbp >> 4) == 0) return 0;
    return (n->cbf_dc >> (1 + uv)) & 1;
}
static int cbf_term_cac(const jmo_cabmbi *n, int cur_intra, int uv, int k) {   /* k: A/B's block (2x2 raster) */
    if (!n) return cur_intra;
    if (n->skip || (n->cbp >> 4) != 2) return 0;
    return (n->cbfc[uv] >> k) & 1;
}

/* ---- residual_block_cabac (7.3.5.3.3) ----------------------------------------------------- */
/* coef[0..n) in scan order; ctxBlockCat cat (Table 9-42), cbf_inc the coded_block_flag's ctxIdxInc
   (ignored for cat 5: 4:2:0 infers that flag); returns coded_block_flag */
static int residual(jmo_cab *e, const int16_t *coef, int n, int cat, int cbf_inc) {
    static const int sig_cat[5] = {0, 15, 29, 44, 47}, abs_cat[5] = {0, 10, 20, 30, 39};
    int nz = 0;
    for (int i = 0; i < n; i++) nz += coef[i] != 0;
    if (cat != 5) jmo_cab_decision(e, 85 + 4 * cat + cbf_inc, nz > 0);
    if (!nz) return 0;
    const int sig_ctx = cat == 5 ? 402 : 105 + sig_cat[cat], last_ctx = cat == 5 ? 417 : 166 + sig_cat[cat];
    const int abs_ctx = cat == 5 ? 426 : 227 + abs_cat[cat];
    /* significance map: significant_coeff_flag, last_significant_coeff_flag up to the last one */
    int left = nz;
    for (int i = 0; i < n - 1; i++) {
        int inc_s, inc_l;
        if (cat == 5) { inc_s = jmo_sig8x8_inc[i]; inc_l = jmo_last8x8_inc[i]; }
        else if (cat == 3) inc_s = inc_l = i < 2 ? i : 2;   /* Min(numDecod / NumC8x8, 2), NumC8x8 = 1 */
        else inc_s = inc_l = i;
        const int sig = coef[i] != 0;
        jmo_cab_decision(e, sig_ctx + inc_s, sig);
        if (sig) {
            left--;
            jmo_cab_decision(e, last_ctx + inc_l, left == 0);
            if (left == 0) break;
        }
    }
    /* levels in reverse scanning order: coeff_abs_level_minus1 (UEG0, uCoff 14), coeff_sign_flag */
    int eq1 = 0, gt1 = 0;
    for (int i = n - 1; i >= 0; i--) {
        if (!coef[i]) continue;
        const int a = (coef[i] < 0 ? -coef[i] : coef[i]) - 1;
        jmo_cab_decision(e, abs_ctx + (gt1 != 0 ? 0 : (1 + eq1 < 4 ? 1 + eq1 : 4)), a > 0);
        if (a > 0) {
            const int ctx = abs_ctx + 5 + (gt1 < 4 - (cat == 3) ? gt1 : 4 - (cat == 3));
            const int pre = a < 14 ? a : 14;
            for (int b = 1; b < pre; b++) jmo_cab_decision(e, ctx, 1);
            if (a < 14) jmo_cab_decision(e, ctx, 0);
            else eg_bypass(e, (unsigned)(a - 14), 0);
        }
        jmo_cab_bypass(e, coef[i] < 0);
        if (a == 0) eq1++;
        else gt1++;
    }
    return 1;
}

/* ---- mvd_l0 (UEG3, signedValFlag 1, uCoff 9; 9.3.3.1.1.7) ------------------------------------ */
static int mvd_abs_left(const jmo_cabnb *nb, const int16_t (*cur)[2], int x4, int y4, int comp) {
    const int v = x4 > 0 ? cur[y4 * 4 + x4 - 1][comp] : nb->A ? nb->mvdA[y4][comp] : 0;
    return v < 0 ? -v : v;
}
static int mvd_abs_up(const jmo_cabnb *nb, const int16_t (*cur)[2], int x4, int y4, int comp) {
    const int v = y4 > 0 ? cur[(y4 - 1) * 4 + x4][comp] : nb->B ? nb->mvdB[x4][comp] : 0;
    return v < 0 ? -v : v;
}
static void mvd_comp(jmo_cab *e, int v, int absum, int comp) {
    const int off = comp ? 47 : 40, a = v < 0 ? -v : v, pre = a < 9 ? a : 9;
    for (int b = 0; b <= pre && b < 9; b++) {
        const int inc = b == 0 ? (absum < 3 ? 0 : absum <= 32 ? 1 : 2) : b < 4 ? b + 2 : 6;
        jmo_cab_decision(e, off + inc, b < pre);
    }
    if (a >= 9) eg_bypass(e, (unsigned)(a - 9), 3);
    if (a) jmo_cab_bypass(e, v < 0);
}
/* the mvd of the (sub-)partition whose top-left 4x4 is (x4, y4) and size w4 x h4; cur[] holds the
   mvds of the current macroblock's partitions coded so far and receives this one */
static void mvd_part(jmo_cab *e, const jmo_cabnb *nb, int16_t (*cur)[2], int x4, int y4, int w4, int h4, int dx, int dy) {
    for (int comp = 0; comp < 2; comp++)
        mvd_comp(e, comp ? dy : dx, mvd_abs_left(nb, (const int16_t(*)[2])cur, x4, y4, comp) +
                                        mvd_abs_up(nb, (const int16_t(*)[2])cur, x4, y4, comp), comp);
    for (int y = y4; y < y4 + h4; y++)
        for (int x = x4; x < x4 + w4; x++) { cur[y * 4 + x][0] = (int16_t)dx; cur[y * 4 + x][1] = (int16_t)dy; }
}

/* sub_mb_type in P slices (Table 9-38 binarisation, ctxIdx 21..23) */
static void sub_mb_type(jmo_cab *e, int sm) {
    switch (sm) {
    case JMH_SMB8x8: jmo_cab_decision(e, 21, 1); break;                                     /* "1"   */
    case JMH_SMB8x4: jmo_cab_decision(e, 21, 0); jmo_cab_decision(e, 22, 0); break;          /* "00"  */
    case JMH_SMB4x8: jmo_cab_decision(e, 21, 0); jmo_cab_decision(e, 22, 1); jmo_cab_decision(e, 23, 1); break; /* "011" */
    default:         jmo_cab_decision(e, 21, 0); jmo_cab_decision(e, 22, 1); jmo_cab_decision(e, 23, 0); break; /* "010" */
    }
}
/* prev_intra4x4/8x8_pred_mode_flag (ctxIdx 68) and rem_intra_pred_mode (FL 3 bins LSB first, 69) */
static void intra_pred_mode(jmo_cab *e, int code) {
    jmo_cab_decision(e, 68, code < 0);
    if (code >= 0)
        for (int b = 0; b < 3; b++) jmo_cab_decision(e, 69, (code >> b) & 1);
}
/* coded_block_pattern luma bin b8 (9.3.3.1.1.4): condTermFlagN = 0 when N is unavailable or its 8x8
   block codes luma (inside the current MB: the bins coded so far), else 1 */
static void cbp_luma_bin(jmo_cab *e, const jmo_cabnb *nb, int cbpl_cur, int b8, int bit) {
    int ta, tb;
    if (b8 & 1) ta = !((cbpl_cur >> (b8 - 1)) & 1);
    else ta = nb->A ? !((nb->A->cbp >> (b8 + 1)) & 1) : 0;
    if (b8 & 2) tb = !((cbpl_cur >> (b8 - 2)) & 1);
    else tb = nb->B ? !((nb->B->cbp >> (b8 + 2)) & 1) : 0;
    jmo_cab_decision(e, 73 + ta + 2 * tb, bit);
}

/* ---- macroblock_layer (7.3.5) of a coded macroblock ----------------------------------------- */
void jmo_cab_skip(jmo_cab *e, const jmo_cabnb *nb) {        /* mb_skip_flag = 1 (9.3.3.1.1.1) */
    jmo_cab_decision(e, 11 + avail_coded(nb->A) + avail_coded(nb->B), 1);
}

void jmo_cab_mb(jmo_cab *e, const jmo_cabnb *nb, const jmo_cabsyn *m, int slice_p, int t8mode, jmo_cabmbi *out,
                int16_t mvd_out[16][2]) {
    const int t = m->mb_type;
    const int i16 = t == JMH_I16MB, nxn = t == JMH_I4MB || t == JMH_I8MB, intra = i16 || nxn;
    const int cbpl = m->cbp & 15, cbpc = m->cbp >> 4;
    jmo_cabmbi me;
    memset(&me, 0, sizeof(me));
    me.intra = (uint8_t)intra; me.i16 = (uint8_t)i16; me.nxn = (uint8_t)nxn;
    me.cbp = (uint8_t)m->cbp;
    int16_t mvd[16][2];
    memset(mvd, 0, sizeof(mvd));

    if (slice_p) jmo_cab_decision(e, 11 + avail_coded(nb->A) + avail_coded(nb->B), 0);
    /* mb_type: Tables 9-36 / 9-37 (9.3.2.5), contexts Table 9-39 */
    if (!slice_p || intra) {
        int off;
        if (slice_p) { jmo_cab_decision(e, 14, 1); off = 17; }     /* prefix "1": intra in a P slice */
        else off = 3;
        if (slice_p) jmo_cab_decision(e, off, i16);
        else jmo_cab_decision(e, off + (nb->A && !nb->A->nxn) + (nb->B && !nb->B->nxn), i16);
        if (i16) {   /* suffix of I_16x16_<mode>_<chroma>_<luma>: terminate, luma, chroma (, 2), mode */
            jmo_cab_terminate(e, 0);
            jmo_cab_decision(e, slice_p ? off + 1 : off + 3, cbpl != 0);
            jmo_cab_decision(e, slice_p ? off + 2 : off + 4, cbpc != 0);
            if (cbpc) jmo_cab_decision(e, slice_p ? off + 2 : off + 5, cbpc == 2);
            jmo_cab_decision(e, slice_p ? off + 3 : off + 6, (m->i16mode >> 1) & 1);
            jmo_cab_decision(e, slice_p ? off + 3 : off + 7, m->i16mode & 1);
        }
    } else {
        jmo_cab_decision(e, 14, 0);
        switch (t) {
        case JMH_P16x16: jmo_cab_decision(e, 15, 0); jmo_cab_decision(e, 16, 0); break;   /* "000" */
        case JMH_P16x8:  jmo_cab_decision(e, 15, 1); jmo_cab_decision(e, 17, 1); break;   /* "011" */
        case JMH_P8x16:  jmo_cab_decision(e, 15, 1); jmo_cab_decision(e, 17, 0); break;   /* "010" */
        default:         jmo_cab_decision(e, 15, 0); jmo_cab_decision(e, 16, 1); break;   /* "001" P_8x8 */
        }
    }
    if (t == JMH_P8x8)
        for (int b8 = 0; b8 < 4; b8++) sub_mb_type(e, m->b8mode[b8]);
    if (nxn && t8mode) {                                     /* transform_size_8x8_flag (9.3.3.1.1.10) */
        jmo_cab_decision(e, 399 + (nb->A && nb->A->t8) + (nb->B && nb->B->t8), t == JMH_I8MB);
        me.t8 = (uint8_t)(t == JMH_I8MB);
    }
    if (t == JMH_I4MB)                                       /* luma4x4BlkIdx order */
        for (int blk = 0; blk < 16; blk++) {
            const int x4 = (blk >> 2 & 1) * 2 + (blk & 1), y4 = (blk >> 3) * 2 + (blk >> 1 & 1);
            intra_pred_mode(e, m->ipm[y4 * 4 + x4]);
        }
    if (t == JMH_I8MB)
        for (int b8 = 0; b8 < 4; b8++) intra_pred_mode(e, m->ipm[(b8 >> 1) * 8 + (b8 & 1) * 2]);
    if (intra) {                                             /* intra_chroma_pred_mode (TU, cMax 3) */
        const int ia = nb->A && nb->A->intra && nb->A->cmode != 0, ib = nb->B && nb->B->intra && nb->B->cmode != 0;
        jmo_cab_decision(e, 64 + ia + ib, m->cmode > 0);
        if (m->cmode > 0) jmo_cab_decision(e, 67, m->cmode > 1);
        if (m->cmode > 1) jmo_cab_decision(e, 67, m->cmode > 2);
        me.cmode = (uint8_t)m->cmode;
    } else if (t == JMH_P8x8) {                              /* sub_mb_pred: mvds per sub-partition */
        for (int b8 = 0; b8 < 4; b8++) {
            const int sm = m->b8mode[b8], w4 = sm == JMH_SMB8x8 || sm == JMH_SMB8x4 ? 2 : 1;
            const int h4 = sm == JMH_SMB8x8 || sm == JMH_SMB4x8 ? 2 : 1;
            for (int y = 0; y < 2; y += h4)
                for (int x = 0; x < 2; x += w4) {
                    const int x4 = (b8 & 1) * 2 + x, y4 = (b8 >> 1) * 2 + y;
                    mvd_part(e, nb, mvd, x4, y4, w4, h4, m->mvd[y4 * 4 + x4][0], m->mvd[y4 * 4 + x4][1]);
                }
        }
    } else {                                                 /* mb_pred: one mvd per partition */
        const int np = t == JMH_P16x16 ? 1 : 2;
        for (int p = 0; p < np; p++) {
            const int x4 = t == JMH_P8x16 ? 2 * p : 0, y4 = t == JMH_P16x8 ? 2 * p : 0;
            mvd_part(e, nb, mvd, x4, y4, t == JMH_P8x16 ? 2 : 4, t == JMH_P16x8 ? 2 : 4, m->mvd[y4 * 4 + x4][0],
                     m->mvd[y4 * 4 + x4][1]);
        }
    }
    if (!i16) {                                              /* coded_block_pattern: FL luma + TU chroma */
        for (int b8 = 0; b8 < 4; b8++) cbp_luma_bin(e, nb, cbpl, b8, (cbpl >> b8) & 1);
        const int ca = nb->A && !nb->A->skip && (nb->A->cbp >> 4) != 0, cb = nb->B && !nb->B->skip && (nb->B->cbp >> 4) != 0;
        jmo_cab_decision(e, 77 + ca + 2 * cb, cbpc != 0);
        if (cbpc) {
            const int ca2 = nb->A && !nb->A->skip && (nb->A->cbp >> 4) == 2, cb2 = nb->B && !nb->B->skip && (nb->B->cbp >> 4) == 2;
            jmo_cab_decision(e, 81 + ca2 + 2 * cb2, cbpc == 2);
        }
        /* transform_size_8x8_flag of an inter macroblock (noSubMbPartSizeLessThan8x8Flag) */
        int no_sub8 = t != JMH_P8x8 || (m->b8mode[0] == JMH_SMB8x8 && m->b8mode[1] == JMH_SMB8x8 &&
                                        m->b8mode[2] == JMH_SMB8x8 && m->b8mode[3] == JMH_SMB8x8);
        if (!intra && cbpl && t8mode && no_sub8) {
            jmo_cab_decision(e, 399 + (nb->A && nb->A->t8) + (nb->B && nb->B->t8), m->t8 != 0);
            me.t8 = (uint8_t)(m->t8 != 0);
        }
    }
    if (cbpl || cbpc || i16) {
        jmo_cab_decision(e, 60, 0);                          /* mb_qp_delta = 0 (no preceding non-zero one) */
        if (i16) {                                           /* Intra16x16DCLevel: cat 0 */
            const int ta = !nb->A ? 1 : nb->A->i16 ? nb->A->cbf_dc & 1 : 0;
            const int tb = !nb->B ? 1 : nb->B->i16 ? nb->B->cbf_dc & 1 : 0;
            me.cbf_dc |= (uint8_t)residual(e, m->luma_dc, 16, 0, ta + 2 * tb);
        }
        for (int b8 = 0; b8 < 4; b8++) {
            if (!((cbpl >> b8) & 1)) continue;
            if (me.t8) {                                     /* residual_block(i8x8): cat 5, 8x8 zig-zag */
                int16_t lv[64];
                for (int j = 0; j < 4; j++) {                /* undo the CAVLC interleave of jmh_mb_result */
                    const int x4 = (b8 & 1) * 2 + (j & 1), y4 = (b8 >> 1) * 2 + (j >> 1);
                    for (int k = 0; k < 16; k++) lv[4 * k + j] = m->luma[y4 * 4 + x4][k];
                }
                residual(e, lv, 64, 5, 0);
                for (int j = 0; j < 4; j++) me.cbf4 |= (uint16_t)(1 << (((b8 >> 1) * 2 + (j >> 1)) * 4 + (b8 & 1) * 2 + (j & 1)));
                continue;
            }
            for (int i4 = 0; i4 < 4; i4++) {
                const int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
                const int ta = x4 ? (me.cbf4 >> (y4 * 4 + x4 - 1)) & 1 : cbf_term_luma(nb->A, intra, 3, y4);
                const int tb = y4 ? (me.cbf4 >> ((y4 - 1) * 4 + x4)) & 1 : cbf_term_luma(nb->B, intra, x4, 3);
                const int16_t *lv = m->luma[y4 * 4 + x4];
                const int f = i16 ? residual(e, lv + 1, 15, 1, ta + 2 * tb) : residual(e, lv, 16, 2, ta + 2 * tb);
                me.cbf4 |= (uint16_t)(f << (y4 * 4 + x4));
            }
        }
        if (cbpc)
            for (int uv = 0; uv < 2; uv++) {                 /* chroma DC: cat 3 */
                const int ta = cbf_term_cdc(nb->A, intra, uv), tb = cbf_term_cdc(nb->B, intra, uv);
                me.cbf_dc |= (uint8_t)(residual(e, m->cdc[uv], 4, 3, ta + 2 * tb) << (1 + uv));
            }
        if (cbpc == 2)
            for (int uv = 0; uv < 2; uv++)                   /* chroma AC: cat 4 */
                for (int k = 0; k < 4; k++) {
                    const int bx = k & 1, by = k >> 1;
                    const int ta = bx ? (me.cbfc[uv] >> (k - 1)) & 1 : cbf_term_cac(nb->A, intra, uv, k + 1);
                    const int tb = by ? (me.cbfc[uv] >> (k - 2)) & 1 : cbf_term_cac(nb->B, intra, uv, k + 2);
                    me.cbfc[uv] |= (uint8_t)(residual(e, m->cac[uv][k] + 1, 15, 4, ta + 2 * tb) << k);
                }
    }
    if (out) *out = me;
    if (mvd_out) memcpy(mvd_out, mvd, sizeof(mvd));
}

/* ---- the partial codings of JM's sub-decisions ---------------------------------------------- */
/* RDCost_for_8x8blocks (CABAC, docs/JM_SEMANTICS.md item 56): sub_mb_type, the sub-partitions'
   mvds, the block's coded_block_pattern bit and, when it keeps coefficients, its four luma 4x4
   residuals, on the running state of the macroblock (cur: the decided blocks), which it advances */
void jmo_cab_b8(jmo_cab *e, const jmo_cabnb *nb, jmo_cabcur *cur, int b8, int sm, const int16_t (*mvd4)[2], int coded,
                const int16_t (*lev4)[16]) {
    sub_mb_type(e, sm);
    const int w4 = sm == JMH_SMB8x8 || sm == JMH_SMB8x4 ? 2 : 1, h4 = sm == JMH_SMB8x8 || sm == JMH_SMB4x8 ? 2 : 1;
    for (int y = 0; y < 2; y += h4)
        for (int x = 0; x < 2; x += w4)
            mvd_part(e, nb, cur->mvd, (b8 & 1) * 2 + x, (b8 >> 1) * 2 + y, w4, h4, mvd4[2 * y + x][0], mvd4[2 * y + x][1]);
    cbp_luma_bin(e, nb, cur->cbpl, b8, coded != 0);
    if (!coded) return;
    cur->cbpl |= (uint8_t)(1 << b8);
    for (int i4 = 0; i4 < 4; i4++) {
        const int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
        const int ta = x4 ? (cur->cbf4 >> (y4 * 4 + x4 - 1)) & 1 : cbf_term_luma(nb->A, 0, 3, y4);
        const int tb = y4 ? (cur->cbf4 >> ((y4 - 1) * 4 + x4)) & 1 : cbf_term_luma(nb->B, 0, x4, 3);
        cur->cbf4 |= (uint16_t)(residual(e, lev4[i4], 16, 2, ta + 2 * tb) << (y4 * 4 + x4));
    }
}
/* RDCost_for_4x4IntraBlocks (item 55): the block's pred-mode syntax and its residual from the state
   at the macroblock start (the current macroblock's own blocks carry no coded_block_flag) */
void jmo_cab_i4(jmo_cab *e, const jmo_cabnb *nb, int x4, int y4, int code, const int16_t *lev) {
    intra_pred_mode(e, code);
    const int ta = x4 ? 0 : cbf_term_luma(nb->A, 1, 3, y4), tb = y4 ? 0 : cbf_term_luma(nb->B, 1, x4, 3);
    residual(e, lev, 16, 2, ta + 2 * tb);
}
/* RDCost_for_8x8IntraBlocks (item 63): the 8x8 block's pred-mode syntax and its luma 8x8 residual
   (ctxBlockCat 5, 8x8 zig-zag order, no coded_block_flag) from the state at the macroblock start */
void jmo_cab_i8(jmo_cab *e, int code, const int16_t *lev64) {
    intra_pred_mode(e, code);
    residual(e, lev64, 64, 5, 0);
}
