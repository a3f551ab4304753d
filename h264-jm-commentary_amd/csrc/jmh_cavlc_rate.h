/*
 * jmh_cavlc_rate.h -- the CAVLC rate of macroblock candidates for RDOptimization = 1 with
 * SymbolMode = 0 (row f4, docs/JM_SEMANTICS.md item 64): JM's RD loop [J] counts what
 * writeMBLayer / writeMotionInfo2NAL / writeCBPandLumaCoeff / writeChromaCoeff (macroblock.c,
 * vlc.c) emit for a candidate.  Those are code lengths only: ue(v) / se(v) / me(v) (9.1, Table 9-4)
 * and residual_block_cavlc (9.2: coeff_token by nC, trailing-ones signs, level_prefix /
 * level_suffix with the suffixLength adaptation and the level_prefix >= 15 escapes, total_zeros,
 * run_before).  No coder state: a candidate's rate depends on its syntax, the TotalCoeff of the
 * neighbouring 4x4 blocks (nC) and the slice's pending mb_skip_run.
 *
 * Written in the common subset of C99 and HIP C++ (the RD kernels of jmh_rdo.hip and the host).
 * tests/test_rate_xcheck.py checks it candidate by candidate against the oracle's own count
 * (oracle/cavlc_bits.c); the product's writer (host/bitstream.c) checks every chosen macroblock's
 * rate against the bits it writes.
 *
 * Reference: /root/reference holds only README.md:1-4 ([J] = JM 8.6 names).
 */
#ifndef JMH_CAVLC_RATE_H
#define JMH_CAVLC_RATE_H

#include <stdint.h>
#include "jmh_cabac_rate.h"   /* jmr_cand, jmr_mbinfo (tcr / tcb), jmr_cur (tc) */

#if defined(__HIPCC__)
#define JMV_FN __host__ __device__ static inline
#define JMV_TABLE static __constant__ const
#define JMV_UNROLL _Pragma("unroll")
#else
#define JMV_FN static inline
#define JMV_TABLE static const
#define JMV_UNROLL
#endif

/* coeff_token lengths (Table 9-5): [nC class 0..2][TrailingOnes][TotalCoeff]; chroma DC (nC -1) */
JMV_TABLE uint8_t jmv_ct[3][4][17] = {
    {{1, 6, 8, 9, 10, 11, 13, 13, 13, 14, 14, 15, 15, 16, 16, 16, 16}, {0, 2, 6, 8, 9, 10, 11, 13, 13, 14, 14, 15, 15, 15, 16, 16, 16},
     {0, 0, 3, 7, 8, 9, 10, 11, 13, 13, 14, 14, 15, 15, 16, 16, 16}, {0, 0, 0, 5, 6, 7, 8, 9, 10, 11, 13, 14, 14, 15, 15, 16, 16}},
    {{2, 6, 6, 7, 8, 8, 9, 11, 11, 12, 12, 12, 13, 13, 13, 14, 14}, {0, 2, 5, 6, 6, 7, 8, 9, 11, 11, 12, 12, 13, 13, 14, 14, 14},
     {0, 0, 3, 6, 6, 7, 8, 9, 11, 11, 12, 12, 13, 13, 13, 14, 14}, {0, 0, 0, 4, 4, 5, 6, 6, 7, 9, 11, 11, 12, 13, 13, 13, 14}},
    {{4, 6, 6, 6, 7, 7, 7, 7, 8, 8, 9, 9, 9, 10, 10, 10, 10}, {0, 4, 5, 5, 5, 5, 6, 6, 7, 8, 8, 9, 9, 9, 10, 10, 10},
     {0, 0, 4, 5, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 10}, {0, 0, 0, 4, 4, 4, 4, 4, 5, 6, 7, 8, 8, 9, 10, 10, 10}}};
JMV_TABLE uint8_t jmv_ctdc[4][5] = {{2, 6, 6, 6, 6}, {0, 1, 6, 7, 8}, {0, 0, 3, 7, 8}, {0, 0, 0, 6, 7}};
/* total_zeros lengths (Tables 9-7, 9-8): [TotalCoeff - 1][total_zeros]; chroma DC (Table 9-9a) */
JMV_TABLE uint8_t jmv_tz[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6}, {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},
    {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5}, {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5}, {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6}, {6, 4, 5, 3, 2, 2, 3, 3, 6}, {6, 6, 4, 2, 2, 3, 2, 5}, {5, 5, 3, 2, 2, 2, 4}, {4, 4, 3, 3, 1, 3},
    {4, 4, 2, 1, 3}, {3, 3, 1, 2}, {2, 2, 1}, {1, 1}};
JMV_TABLE uint8_t jmv_tzdc[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
/* run_before lengths (Table 9-10): [min(zerosLeft, 7) - 1][run_before] */
JMV_TABLE uint8_t jmv_rb[7][15] = {{1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3}, {2, 3, 3, 3, 3, 3, 3},
                                   {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
/* coded_block_pattern -> codeNum (Table 9-4, ChromaArrayType 1): intra (I_NxN), inter */
JMV_TABLE uint8_t jmv_cbp_i[48] = {3,  29, 30, 17, 31, 18, 37, 8,  32, 38, 19, 9,  20, 10, 11, 2,  16, 33, 34, 21, 35, 22, 39, 4,
                                   36, 40, 23, 5,  24, 6,  7,  1,  41, 42, 43, 25, 44, 26, 46, 12, 45, 47, 27, 13, 28, 14, 15, 0};
JMV_TABLE uint8_t jmv_cbp_p[48] = {0,  2,  3,  7,  4,  8,  17, 13, 5,  18, 9,  14, 10, 15, 16, 11, 1,  32, 33, 36, 34, 37, 44, 40,
                                   35, 45, 38, 41, 39, 42, 43, 19, 6,  24, 25, 20, 26, 21, 46, 28, 27, 47, 22, 29, 23, 30, 31, 12};

JMV_FN int jmv_ue(unsigned v) { return 127 - 2 * __builtin_clzll((unsigned long long)v + 1ull); }   /* 2 floor(log2(v+1)) + 1 */
/* P_Skip: 0 bits (the run goes out with the next coded macroblock) except at the picture's last
   macroblock, where JM's writeMBLayer writes the pending run, this macroblock included (item 64(a)) */
JMV_FN int jmv_skip(int skip_run, int last_in_picture) { return last_in_picture ? jmv_ue((unsigned)skip_run + 1u) : 0; }
JMV_FN int jmv_se(int v) { return jmv_ue(v > 0 ? (unsigned)(2 * v - 1) : (unsigned)(-2 * v)); }

/* residual_block_cavlc: coef[st * i] for i in [0, n) in scan order (st 4: a CAVLC-interleaved 4x4
   of an 8x8 block), nC (-1: chroma DC); bits, *tc = TotalCoeff.  The non-zero positions come from
   one bit mask; the levels are visited from the highest frequency */
JMV_FN int jmv_block(const int16_t *coef, int st, int n, int nC, int *tc) {
    uint32_t nzm = 0;
    for (int i = 0; i < n; i++)
        if (coef[st * i]) nzm |= 1u << i;
    const int total = __builtin_popcount(nzm);
    *tc = total;
    int t1 = 0, bits = 0;
    if (total) {                                      /* TrailingOnes: up to three +-1 from the end */
        uint32_t m = nzm;
        while (t1 < 3 && m) {
            const int i = 31 - __builtin_clz(m);
            if (coef[st * i] != 1 && coef[st * i] != -1) break;
            m &= ~(1u << i);
            t1++;
        }
    }
    bits = nC == -1 ? jmv_ctdc[t1][total] : nC >= 8 ? 6 : jmv_ct[nC < 2 ? 0 : nC < 4 ? 1 : 2][t1][total];
    if (!total) return bits;
    bits += t1;
    int sl = total > 10 && t1 < 3;
    uint32_t m = nzm;
    for (int k = 0; k < total; k++) {
        const int i = 31 - __builtin_clz(m);
        m &= ~(1u << i);
        if (k < t1) continue;
        const int v = coef[st * i], a = v < 0 ? -v : v;
        int code = 2 * a - 2 + (v < 0);                       /* levelCode */
        if (k == t1 && t1 < 3) code -= 2;
        if (sl == 0) bits += code < 14 ? code + 1 : code < 30 ? 19 : 0;
        else if (code < (15 << sl)) bits += (code >> sl) + 1 + sl;
        if ((sl == 0 && code >= 30) || (sl > 0 && code >= (15 << sl))) {   /* level_prefix >= 15 */
            int rest = code - (sl == 0 ? 30 : 15 << sl), p = 15;
            while (rest >= (1 << (p - 3))) { rest -= 1 << (p - 3); p++; }
            bits += 2 * p - 2;                                 /* prefix + 1 + (p - 3) suffix bits */
        }
        if (sl == 0) sl = 1;
        if (a > (3 << (sl - 1)) && sl < 6) sl++;
    }
    const int last = 31 - __builtin_clz(nzm), tz = last + 1 - total;
    if (total < n) bits += nC == -1 ? jmv_tzdc[total - 1][tz] : jmv_tz[total - 1][tz];
    int zl = tz, prev = last;
    m = nzm & ~(1u << last);
    while (zl > 0 && m) {                                 /* run_before of all but the lowest one */
        const int i = 31 - __builtin_clz(m);
        const int run = prev - i - 1;
        bits += jmv_rb[zl > 6 ? 6 : zl - 1][run];
        zl -= run;
        prev = i;
        m &= ~(1u << i);
    }
    return bits;
}

/* the neighbours' TotalCoeff the current macroblock's nC reads: A's right column, B's bottom row
   (luma 4, Cb 2, Cr 2), in jmr_mbinfo (jmh_cabac_rate.h: tcr / tcb) */
JMV_FN int jmv_nc(const uint8_t *tcrA, const uint8_t *tcbB, const uint8_t *cur, int comp, int x4, int y4) {
    const int w = comp ? 2 : 4, base = comp ? 16 + 4 * (comp - 1) : 0, nbase = comp ? 4 + 2 * (comp - 1) : 0;
    const int na = x4 ? cur[base + y4 * w + x4 - 1] : tcrA ? tcrA[nbase + y4] : -1;
    const int nb = y4 ? cur[base + (y4 - 1) * w + x4] : tcbB ? tcbB[nbase + x4] : -1;
    return na >= 0 && nb >= 0 ? (na + nb + 1) >> 1 : na >= 0 ? na : nb >= 0 ? nb : 0;
}

/* the luma residual of 8x8 block b8: four 4x4 blocks in coding order (cat: 1 I16 AC, else 2; with
   lev64, an 8x8-transform block, the four CAVLC-interleaved 4x4 of lev64).  cur (read only) holds the
   macroblock's other decided blocks; the block's own four TotalCoeff stay in registers (the loop
   unrolls) and go to tco */
JMV_FN int jmv_luma8(const uint8_t *tcrA, const uint8_t *tcbB, const uint8_t *cur, int b8, const int16_t (*luma)[16], int ac,
                     const int16_t *lev64, uint8_t *tco) {
    int bits = 0, t[4];
JMV_UNROLL
    for (int i4 = 0; i4 < 4; i4++) {
        const int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
        const int na = (i4 & 1) ? t[i4 - 1] : x4 ? cur[y4 * 4 + x4 - 1] : tcrA ? tcrA[y4] : -1;
        const int nb = (i4 & 2) ? t[i4 - 2] : y4 ? cur[(y4 - 1) * 4 + x4] : tcbB ? tcbB[x4] : -1;
        const int nC = na >= 0 && nb >= 0 ? (na + nb + 1) >> 1 : na >= 0 ? na : nb >= 0 ? nb : 0;
        if (lev64) bits += jmv_block(lev64 + i4, 4, 16, nC, &t[i4]);
        else if (ac) bits += jmv_block(luma[y4 * 4 + x4] + 1, 1, 15, nC, &t[i4]);
        else bits += jmv_block(luma[y4 * 4 + x4], 1, 16, nC, &t[i4]);
    }
JMV_UNROLL
    for (int i4 = 0; i4 < 4; i4++) tco[i4] = (uint8_t)t[i4];
    return bits;
}
/* tco of jmv_luma8 into a macroblock's 24 TotalCoeff */
JMV_FN void jmv_put8(uint8_t *cur, int b8, const uint8_t *tco) {
JMV_UNROLL
    for (int i4 = 0; i4 < 4; i4++) cur[((b8 >> 1) * 2 + (i4 >> 1)) * 4 + (b8 & 1) * 2 + (i4 & 1)] = tco[i4];
}
JMV_FN const uint8_t *jmv_tcr(const jmr_mbinfo *n) { return n ? n->tcr : 0; }
JMV_FN const uint8_t *jmv_tcb(const jmr_mbinfo *n) { return n ? n->tcb : 0; }

/* a whole coded macroblock (RDCost_for_macroblocks [J] with CAVLC, item 64): the mb_skip_run before
   it in P slices and macroblock_layer (7.3.5); out (may be NULL): what it leaves for its
   neighbours (kind, cbp and the TotalCoeff of its right column / bottom row); cur: a 24-byte work
   buffer (the macroblock's TotalCoeff: 16 luma raster, 4 Cb, 4 Cr), in LDS or global memory on the
   device so that its run-time indexing stays out of scratch */
JMV_FN int jmv_mb(const jmr_mbinfo *A, const jmr_mbinfo *B, const jmr_cand *r, int slice_p, int t8mode, int skip_run,
                  uint8_t *cur, jmr_mbinfo *out) {
    const int t = r->mb_type, i16 = t == JMH_I16MB, nxn = t == JMH_I4MB || t == JMH_I8MB, intra = i16 || nxn;
    const int cbpl = r->cbp & 15, cbpc = r->cbp >> 4;
    const uint8_t *ta = jmv_tcr(A), *tb = jmv_tcb(B);
    for (int k = 0; k < 24; k++) cur[k] = 0;
    int bits = slice_p ? jmv_ue((unsigned)skip_run) : 0;
    const int mbt = i16 ? 1 + r->i16mode + 4 * cbpc + 12 * (cbpl != 0) : nxn ? 0 : t == JMH_P8x8 ? 3 : t - 1;
    bits += jmv_ue((unsigned)(mbt + 5 * (slice_p && intra)));
    /* the candidate (a private struct on the device) is read at constant indices only: the loops over
       its arrays unroll */
    if (t == JMH_P8x8)
JMV_UNROLL
        for (int b = 0; b < 4; b++) bits += jmv_ue((unsigned)(r->b8mode[b] - 4));
    if (nxn && t8mode) bits++;                             /* transform_size_8x8_flag */
    if (nxn)                                               /* I8MB: the 8x8 blocks' top-left 4x4 */
        for (int q = 0; q < 16; q++)
            if (t == JMH_I4MB || !(q & 5)) bits += r->ipm[q] < 0 ? 1 : 4;
    if (intra) bits += jmv_ue((unsigned)r->cmode);
    else if (t == JMH_P8x8)                                /* mvd_l0 of every sub-partition */
JMV_UNROLL
        for (int b8 = 0; b8 < 4; b8++) {
            const int sm = r->b8mode[b8], w4 = sm == JMH_SMB8x8 || sm == JMH_SMB8x4 ? 2 : 1;
            const int h4 = sm == JMH_SMB8x8 || sm == JMH_SMB4x8 ? 2 : 1;
            for (int y = 0; y < 2; y += h4)
                for (int x = 0; x < 2; x += w4) {
                    const int q = ((b8 >> 1) * 2 + y) * 4 + (b8 & 1) * 2 + x;
                    bits += jmv_se(r->mvd[q][0]) + jmv_se(r->mvd[q][1]);
                }
        }
    else                                                   /* 16x16: one partition; 16x8 / 8x16: two */
        for (int p = 0; p < (t == JMH_P16x16 ? 1 : 2); p++) {
            const int q = t == JMH_P16x8 ? 8 * p : t == JMH_P8x16 ? 2 * p : 0;
            bits += jmv_se(r->mvd[q][0]) + jmv_se(r->mvd[q][1]);
        }
    if (!i16) bits += jmv_ue(intra ? jmv_cbp_i[r->cbp] : jmv_cbp_p[r->cbp]);
    if (!intra && cbpl && t8mode &&
        (t != JMH_P8x8 || (r->b8mode[0] == 4 && r->b8mode[1] == 4 && r->b8mode[2] == 4 && r->b8mode[3] == 4)))
        bits++;                                            /* transform_size_8x8_flag */
    if (cbpl || cbpc || i16) {
        bits++;                                            /* mb_qp_delta = 0 */
        int tt;
        if (i16) bits += jmv_block(r->luma_dc, 1, 16, jmv_nc(ta, tb, cur, 0, 0, 0), &tt);
        for (int b8 = 0; b8 < 4; b8++)
            if ((cbpl >> b8) & 1) {
                uint8_t tco[4];
                bits += jmv_luma8(ta, tb, cur, b8, r->luma, i16, 0, tco);
                jmv_put8(cur, b8, tco);
            }
        if (cbpc)
            for (int uv = 0; uv < 2; uv++) bits += jmv_block(r->cdc[uv], 1, 4, -1, &tt);
        if (cbpc == 2)
            for (int uv = 0; uv < 2; uv++)
                for (int k = 0; k < 4; k++) {
                    bits += jmv_block(r->cac[uv][k] + 1, 1, 15, jmv_nc(ta, tb, cur, 1 + uv, k & 1, k >> 1), &tt);
                    cur[16 + 4 * uv + k] = (uint8_t)tt;
                }
    }
    if (out) {
        jmr_mbinfo mi = {0};
        mi.kind = (uint8_t)(i16 ? JMR_K_I16 : nxn ? JMR_K_INXN : JMR_K_INTER);
        mi.cbp = (uint8_t)r->cbp;
JMV_UNROLL
        for (int i = 0; i < 4; i++) { mi.tcr[i] = cur[4 * i + 3]; mi.tcb[i] = cur[12 + i]; }
JMV_UNROLL
        for (int uv = 0; uv < 2; uv++)
JMV_UNROLL
            for (int i = 0; i < 2; i++) { mi.tcr[4 + 2 * uv + i] = cur[16 + 4 * uv + 2 * i + 1]; mi.tcb[4 + 2 * uv + i] = cur[16 + 4 * uv + 2 + i]; }
        *out = mi;
    }
    return bits;
}
/* RDCost_for_8x8blocks with CAVLC (item 64): sub_mb_type, the sub-partitions' mvds and, when it keeps
   coefficients, its four luma 4x4 residuals; cur (the decided blocks) gains this block's TotalCoeff */
JMV_FN int jmv_b8(const jmr_mbinfo *A, const jmr_mbinfo *B, jmr_cur *cur, int b8, int sm, const int16_t (*mvd4)[2], int coded,
                  const int16_t (*lev4)[16]) {
    int bits = jmv_ue((unsigned)(sm - 4));
    const int w4 = sm == 4 || sm == 5 ? 2 : 1, h4 = sm == 4 || sm == 6 ? 2 : 1;
    for (int y = 0; y < 2; y += h4)
        for (int x = 0; x < 2; x += w4) bits += jmv_se(mvd4[2 * y + x][0]) + jmv_se(mvd4[2 * y + x][1]);
    for (int i4 = 0; i4 < 4; i4++) {
        const int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
        int t = 0;
        if (coded) bits += jmv_block(lev4[i4], 1, 16, jmv_nc(jmv_tcr(A), jmv_tcb(B), cur->tc, 0, x4, y4), &t);
        cur->tc[y4 * 4 + x4] = (uint8_t)t;
    }
    return bits;
}
/* RDCost_for_4x4IntraBlocks with CAVLC: the mode syntax (1 or 4 bits) + the block's residual (nC from
   the macroblock's decided blocks, cur_tc, read only); *tc: the block's TotalCoeff */
JMV_FN int jmv_i4(const jmr_mbinfo *A, const jmr_mbinfo *B, const uint8_t *cur_tc, int x4, int y4, int code, const int16_t *lev,
                  int *tc) {
    return (code < 0 ? 1 : 4) + jmv_block(lev, 1, 16, jmv_nc(jmv_tcr(A), jmv_tcb(B), cur_tc, 0, x4, y4), tc);
}
/* RDCost_for_8x8IntraBlocks with CAVLC: the mode syntax + the block's four interleaved 4x4 residuals;
   tco: their TotalCoeff */
JMV_FN int jmv_i8(const jmr_mbinfo *A, const jmr_mbinfo *B, const uint8_t *cur_tc, int b8, int code, const int16_t *lev64,
                  uint8_t *tco) {
    return (code < 0 ? 1 : 4) + jmv_luma8(jmv_tcr(A), jmv_tcb(B), cur_tc, b8, 0, 0, lev64, tco);
}

#endif
