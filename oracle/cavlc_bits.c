/*
 * cavlc_bits.c — the oracle's CAVLC bit count: the rate of RDOptimization 1 with SymbolMode 0
 * (TEST INFRASTRUCTURE ONLY; see jm_oracle.h for the parity status).
 *
 * JM's RD loop [J] with the UVLC/CAVLC entropy coder takes a candidate's rate as the length of what
 * writeMBLayer / writeMotionInfo2NAL / writeCBPandLumaCoeff / writeChromaCoeff emit for it
 * (macroblock.c, vlc.c).  This file restates those lengths from ITU-T H.264 7.3.5 and 9.1 / 9.2:
 * ue(v) / se(v) / me(v) (Table 9-4) code lengths and residual_block_cavlc (coeff_token by nC, the
 * trailing-ones signs, level_prefix / level_suffix with the suffixLength adaptation and the
 * level_prefix >= 15 escapes, total_zeros, run_before), over the code-length tables of the
 * independent decoder (decoder.c, proven by its closed loop).  Nothing is written: only lengths.
 * It shares no code with the product (csrc/jmh_cavlc_rate.h, host/bitstream.c);
 * tests/test_rate_xcheck.py compares the two on every RD candidate.  The RD choices it serves are
 * docs/JM_SEMANTICS.md item 64.
 */
#include "jmo_internal.h"

static int ue_len(unsigned v) {                            /* 9.1: 2 * floor(log2(v + 1)) + 1 */
    int n = 0;
    for (unsigned x = v + 1; x > 1; x >>= 1) n++;
    return 2 * n + 1;
}
static int se_len(int v) { return ue_len(v > 0 ? (unsigned)(2 * v - 1) : (unsigned)(-2 * v)); }   /* 9.1.1 */

/* residual_block_cavlc (7.3.5.3.2, 9.2): coef[0..n) in scan order, nC (-1: chroma DC); returns the
   block's bits and its TotalCoeff */
int jmo_cavlc_block_bits(const int16_t *coef, int n, int nC, int *total_coeff) {
    int lev[16], pos[16], tc = 0;
    for (int i = n - 1; i >= 0; i--)                       /* levels in reverse scanning order */
        if (coef[i]) { lev[tc] = coef[i]; pos[tc] = i; tc++; }
    *total_coeff = tc;
    int t1 = 0;
    while (t1 < tc && t1 < 3 && (lev[t1] == 1 || lev[t1] == -1)) t1++;
    int bits;                                              /* coeff_token (Table 9-5) */
    if (nC == -1) bits = jmo_ctdc_len[t1][tc];
    else if (nC >= 8) bits = 6;
    else bits = jmo_ct_len[nC < 2 ? 0 : nC < 4 ? 1 : 2][t1][tc];
    if (!tc) return bits;
    bits += t1;                                            /* trailing_ones_sign_flag */
    int sl = tc > 10 && t1 < 3 ? 1 : 0;                    /* suffixLength */
    for (int i = t1; i < tc; i++) {
        const int a = lev[i] < 0 ? -lev[i] : lev[i];
        int code = lev[i] > 0 ? 2 * lev[i] - 2 : -2 * lev[i] - 1;   /* levelCode */
        if (i == t1 && t1 < 3) code -= 2;
        int prefix, ssize;                                 /* level_prefix, levelSuffixSize */
        if (sl == 0 && code < 14) { prefix = code; ssize = 0; }
        else if (sl == 0 && code < 30) { prefix = 14; ssize = 4; }
        else if (sl > 0 && (code >> sl) < 15) { prefix = code >> sl; ssize = sl; }
        else {                                             /* escapes: level_prefix >= 15 */
            int rest = code - (sl == 0 ? 30 : 15 << sl);
            prefix = 15;
            while (rest >= (1 << (prefix - 3))) { rest -= 1 << (prefix - 3); prefix++; }
            ssize = prefix - 3;
        }
        bits += prefix + 1 + ssize;
        if (sl == 0) sl = 1;
        if (a > (3 << (sl - 1)) && sl < 6) sl++;
    }
    const int total_zeros = pos[0] + 1 - tc;
    if (tc < n) bits += nC == -1 ? jmo_tzdc_len[tc - 1][total_zeros] : jmo_tz_len[tc - 1][total_zeros];
    int zl = total_zeros;
    for (int i = 0; i < tc - 1 && zl > 0; i++) {           /* run_before */
        const int run = pos[i] - pos[i + 1] - 1;
        bits += jmo_rb_len[zl > 6 ? 6 : zl - 1][run];
        zl -= run;
    }
    return bits;
}

/* nC of a 4x4 block (9.2.1): comp 0 luma (x4, y4 in 0..3), 1 / 2 chroma (0..1); cur: the current
   macroblock's TotalCoeff so far (jmo_cavnb layout: 16 luma raster, 4 Cb, 4 Cr) */
static int nc_of(const jmo_cavnb *nb, const uint8_t *cur, int comp, int x4, int y4) {
    const int base = comp ? 16 + 4 * (comp - 1) : 0, w = comp ? 2 : 4;
    int na = -1, nbv = -1;
    if (x4 > 0) na = cur[base + y4 * w + x4 - 1];
    else if (nb->A) na = nb->A[base + y4 * w + w - 1];
    if (y4 > 0) nbv = cur[base + (y4 - 1) * w + x4];
    else if (nb->B) nbv = nb->B[base + (w - 1) * w + x4];
    if (na >= 0 && nbv >= 0) return (na + nbv + 1) >> 1;
    return na >= 0 ? na : nbv >= 0 ? nbv : 0;
}
static int cbp_code(int cbp, int intra) {                  /* me(v): the codeNum of Table 9-4 */
    const uint8_t *t = intra ? jmo_cbp_intra : jmo_cbp_inter;
    for (int k = 0; k < 48; k++)
        if (t[k] == cbp) return k;
    return 0;
}

/* the luma residual of 8x8 block b8 (four 4x4 blocks in coding order; an 8x8-transform block as its
   four CAVLC-interleaved 4x4 blocks, 7.3.5.3.2); cat 1 (I16 AC, 15 levels) when ac */
static int luma8_bits(const jmo_cavnb *nb, uint8_t *cur, int b8, const int16_t (*luma)[16], int ac) {
    int bits = 0;
    for (int i4 = 0; i4 < 4; i4++) {
        const int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
        const int16_t *lv = luma[y4 * 4 + x4];
        int t;
        bits += ac ? jmo_cavlc_block_bits(lv + 1, 15, nc_of(nb, cur, 0, x4, y4), &t)
                   : jmo_cavlc_block_bits(lv, 16, nc_of(nb, cur, 0, x4, y4), &t);
        cur[y4 * 4 + x4] = (uint8_t)t;
    }
    return bits;
}

/* a P_Skip candidate: nothing is written for it (its run goes out with the next coded macroblock of
   the slice), except at the picture's last macroblock, where writeMBLayer finds no next macroblock
   (FmoGetNextMBNr -1) and writes the run, this macroblock included: ue(skip_run + 1)
   (docs/JM_SEMANTICS.md item 64(a)) */
int jmo_cavlc_skip_bits(int skip_run, int last_in_picture) {
    return last_in_picture ? ue_len((unsigned)skip_run + 1u) : 0;
}

/* a whole macroblock candidate: the mb_skip_run before it (P slices), macroblock_layer (7.3.5) as
   writeMBLayer writes it; tc_out (may be NULL): its 24 TotalCoeff for the neighbours' nC */
int jmo_cavlc_mb_bits(const jmo_cavnb *nb, const jmo_cabsyn *m, int slice_p, int t8mode, int skip_run, uint8_t tc_out[24]) {
    const int t = m->mb_type, i16 = t == JMH_I16MB, nxn = t == JMH_I4MB || t == JMH_I8MB, intra = i16 || nxn;
    const int cbpl = m->cbp & 15, cbpc = m->cbp >> 4;
    uint8_t cur[24] = {0};
    int bits = slice_p ? ue_len((unsigned)skip_run) : 0;
    int ue_type;                                           /* mb_type (Tables 7-11, 7-13) */
    if (i16) ue_type = 1 + m->i16mode + 4 * cbpc + (cbpl ? 12 : 0);
    else if (nxn) ue_type = 0;
    else ue_type = t == JMH_P8x8 ? 3 : t - 1;
    bits += ue_len((unsigned)(ue_type + (slice_p && intra ? 5 : 0)));
    if (t == JMH_P8x8)
        for (int b8 = 0; b8 < 4; b8++) bits += ue_len((unsigned)(m->b8mode[b8] - 4));   /* sub_mb_type (Table 7-17) */
    if (nxn && t8mode) bits += 1;                          /* transform_size_8x8_flag */
    if (t == JMH_I4MB)
        for (int q = 0; q < 16; q++) bits += m->ipm[q] < 0 ? 1 : 4;
    if (t == JMH_I8MB)
        for (int b8 = 0; b8 < 4; b8++) bits += m->ipm[(b8 >> 1) * 8 + (b8 & 1) * 2] < 0 ? 1 : 4;
    if (intra) bits += ue_len((unsigned)m->cmode);         /* intra_chroma_pred_mode */
    else if (t == JMH_P8x8)                                /* mvd_l0 of every (sub-)partition */
        for (int b8 = 0; b8 < 4; b8++) {
            const int sm = m->b8mode[b8], w4 = sm == JMH_SMB8x8 || sm == JMH_SMB8x4 ? 2 : 1;
            const int h4 = sm == JMH_SMB8x8 || sm == JMH_SMB4x8 ? 2 : 1;
            for (int y = 0; y < 2; y += h4)
                for (int x = 0; x < 2; x += w4) {
                    const int q = ((b8 >> 1) * 2 + y) * 4 + (b8 & 1) * 2 + x;
                    bits += se_len(m->mvd[q][0]) + se_len(m->mvd[q][1]);
                }
        }
    else
        for (int p = 0; p < (t == JMH_P16x16 ? 1 : 2); p++) {
            const int q = (t == JMH_P16x8 ? 2 * p : 0) * 4 + (t == JMH_P8x16 ? 2 * p : 0);
            bits += se_len(m->mvd[q][0]) + se_len(m->mvd[q][1]);
        }
    if (!i16) bits += ue_len((unsigned)cbp_code(m->cbp, intra));   /* coded_block_pattern me(v) */
    const int no_sub8 = t != JMH_P8x8 || (m->b8mode[0] == JMH_SMB8x8 && m->b8mode[1] == JMH_SMB8x8 &&
                                          m->b8mode[2] == JMH_SMB8x8 && m->b8mode[3] == JMH_SMB8x8);
    if (!intra && cbpl && t8mode && no_sub8) bits += 1;    /* transform_size_8x8_flag */
    if (cbpl || cbpc || i16) {
        bits += se_len(0);                                 /* mb_qp_delta */
        int tcdc;
        if (i16) bits += jmo_cavlc_block_bits(m->luma_dc, 16, nc_of(nb, cur, 0, 0, 0), &tcdc);
        for (int b8 = 0; b8 < 4; b8++)
            if ((cbpl >> b8) & 1) bits += luma8_bits(nb, cur, b8, m->luma, i16);
        if (cbpc)
            for (int uv = 0; uv < 2; uv++) bits += jmo_cavlc_block_bits(m->cdc[uv], 4, -1, &tcdc);
        if (cbpc == 2)
            for (int uv = 0; uv < 2; uv++)
                for (int k = 0; k < 4; k++) {
                    int tk;
                    bits += jmo_cavlc_block_bits(m->cac[uv][k] + 1, 15, nc_of(nb, cur, 1 + uv, k & 1, k >> 1), &tk);
                    cur[16 + 4 * uv + k] = (uint8_t)tk;
                }
    }
    if (tc_out) memcpy(tc_out, cur, 24);
    return bits;
}

/* RDCost_for_8x8blocks with CAVLC (item 64): sub_mb_type, the sub-partitions' mvds and, when it keeps
   coefficients, the block's four luma 4x4 residuals (nC from the decided blocks, cur->tc) */
int jmo_cavlc_b8_bits(const jmo_cavnb *nb, uint8_t cur_tc[24], int b8, int sm, const int16_t (*mvd4)[2], int coded,
                      const int16_t (*lev4)[16]) {
    int bits = ue_len((unsigned)(sm - 4));
    const int w = sm == JMH_SMB8x8 || sm == JMH_SMB8x4 ? 2 : 1, h = sm == JMH_SMB8x8 || sm == JMH_SMB4x8 ? 2 : 1;
    for (int y = 0; y < 2; y += h)
        for (int x = 0; x < 2; x += w) bits += se_len(mvd4[2 * y + x][0]) + se_len(mvd4[2 * y + x][1]);
    for (int i4 = 0; i4 < 4; i4++) {
        const int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
        int t = 0;
        if (coded) bits += jmo_cavlc_block_bits(lev4[i4], 16, nc_of(nb, cur_tc, 0, x4, y4), &t);
        cur_tc[y4 * 4 + x4] = (uint8_t)t;
    }
    return bits;
}
/* RDCost_for_4x4IntraBlocks with CAVLC (item 64): the mode syntax (1 or 4 bits) and the block's
   residual (nC from the macroblock's decided blocks, cur_tc); sets cur_tc of the block */
int jmo_cavlc_i4_bits(const jmo_cavnb *nb, uint8_t cur_tc[24], int x4, int y4, int code, const int16_t *lev) {
    int t;
    const int bits = (code < 0 ? 1 : 4) + jmo_cavlc_block_bits(lev, 16, nc_of(nb, cur_tc, 0, x4, y4), &t);
    cur_tc[y4 * 4 + x4] = (uint8_t)t;
    return bits;
}
/* RDCost_for_8x8IntraBlocks with CAVLC: the mode syntax and the block's four interleaved 4x4 residuals
   (lev64 in 8x8 zig-zag order) */
int jmo_cavlc_i8_bits(const jmo_cavnb *nb, uint8_t cur_tc[24], int b8, int code, const int16_t *lev64) {
    int16_t il[16][16];
    memset(il, 0, sizeof(il));
    for (int j = 0; j < 4; j++) {
        const int x4 = (b8 & 1) * 2 + (j & 1), y4 = (b8 >> 1) * 2 + (j >> 1);
        for (int k = 0; k < 16; k++) il[y4 * 4 + x4][k] = lev64[4 * k + j];
    }
    return (code < 0 ? 1 : 4) + luma8_bits(nb, cur_tc, b8, (const int16_t(*)[16])il, 0);
}
