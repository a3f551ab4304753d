/*
 * jmh_cabac_rate.h -- the CABAC rate of macroblock candidates for RDOptimization = 1 (row f4):
 * JM lencod's RD loop [J] codes every candidate with the real arithmetic coder between
 * store_coding_state / reset_coding_state (rdopt_coding_state.c) and takes
 *     rate = arienco_bits_written(after) - arienco_bits_written(before)        (biariencode.c)
 * (8 * bytes + 8 - Ebits_to_go + Ebits_to_follow).  Each renormalisation step of 9.3.4.2 either
 * emits one bit (with the outstanding ones) or adds one outstanding bit, and a bypass bin one
 * step: so that count grows by exactly one per step, whatever codIOffset holds.  The rate is
 * therefore a function of codIRange and the context states alone, and this engine tracks only
 * those (no codIOffset, no bytes): bits = renormalisation steps + bypass bins.
 *
 * Binarisations and ctxIdx selection restate host/cabac.c (the product's slice writer, checked
 * against the independent decoder oracle/decoder.c) over a dense context index space (JMR_CTX),
 * written in the common subset of C99 and HIP C++ so that the same text is the RD rate of the
 * CPU oracle (oracle/rdo.c) and of the device (k_mb_rdo, jmh_rdo.hip).  tests/test_rdo.py checks
 * that the rate of every committed macroblock equals the bits host/cabac.c writes for it.
 *
 * Reference: /root/reference holds only README.md:1-4, so no JM file:line exists ([J] = JM 8.6
 * names); docs/JM_SEMANTICS.md items 53-60 pin the RD choices.
 */
#ifndef JMH_CABAC_RATE_H
#define JMH_CABAC_RATE_H

#include <stdint.h>
#include "../../include/jmhip.h"

#if defined(__HIPCC__)
#define JMR_FN __host__ __device__ static inline
#define JMR_TABLE static __constant__ const
#else
#define JMR_FN static inline
#define JMR_TABLE static const
#endif

/* dense context index of spec ctxIdx i (the contexts this encoder codes, tools/gen_cabac_tables.py) */
#define JMR_CTX(i) ((i) < 24 ? (i) : (i) < 54 ? (i) - 16 : (i) < 70 ? (i) - 22 : (i) < 276 ? (i) - 25 : (i) - 148)
#define JMR_NCTX 288

#include "jmh_cabac_tables.h"

/* Table 9-44: rangeTabLPS, transIdxLPS */
JMR_TABLE uint8_t jmr_lps[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205}, {116, 142, 169, 195},
    {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166}, {95, 116, 137, 158},  {90, 110, 130, 150},
    {85, 104, 123, 142},  {81, 99, 117, 135},   {77, 94, 111, 128},   {73, 89, 105, 122},   {69, 85, 100, 116},
    {66, 80, 95, 110},    {62, 76, 90, 104},    {59, 72, 86, 99},     {56, 69, 81, 94},     {53, 65, 77, 89},
    {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},     {41, 50, 59, 69},
    {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},     {33, 41, 48, 56},     {32, 39, 46, 53},
    {30, 37, 43, 50},     {29, 35, 41, 48},     {27, 33, 39, 45},     {26, 31, 37, 43},     {24, 30, 35, 41},
    {23, 28, 33, 39},     {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},     {19, 23, 27, 31},
    {18, 22, 26, 30},     {17, 21, 25, 28},     {16, 20, 23, 27},     {15, 19, 22, 25},     {14, 18, 21, 24},
    {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},     {12, 14, 17, 20},     {11, 14, 16, 19},
    {11, 13, 15, 18},     {10, 12, 15, 17},     {10, 12, 14, 16},     {9, 11, 13, 15},      {9, 11, 12, 14},
    {8, 10, 12, 14},      {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},       {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2}};
JMR_TABLE uint8_t jmr_trans_lps[64] = {
    0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12, 13, 13, 15, 15, 16, 16,
    18, 18, 19, 19, 21, 21, 22, 22, 23, 24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30,
    31, 32, 32, 33, 33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};
JMR_TABLE uint8_t jmr_sig8x8_inc[63] = {0,  1,  2,  3,  4,  5,  5,  4,  4,  3,  3,  4,  4,  4,  5,  5,  4,  4,  4,  4,  3,
                                        3,  6,  7,  7,  7,  8,  9,  10, 9,  8,  7,  7,  6,  11, 12, 13, 11, 6,  7,  8,  9,
                                        14, 10, 9,  8,  6,  11, 12, 13, 11, 6,  9,  14, 10, 9,  11, 12, 13, 11, 14, 10, 12};
JMR_TABLE uint8_t jmr_last8x8_inc[63] = {0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2,
                                         2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4,
                                         4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7, 8, 8, 8};

/* ---- engine: context states (state << 1 | valMPS) + codIRange + the bit count ------------- */
typedef struct jmr_eng {
    uint8_t *st;          /* JMR_NCTX contexts                                                  */
    uint32_t range;       /* codIRange, 256..510 between bins                                  */
    int32_t bits;         /* arienco_bits_written delta (renormalisation steps + bypass bins)   */
} jmr_eng;

/* 9.3.1.1 with slice QP SliceQPY (cabac_init_idc 0 in P slices): context i, and all of them */
JMR_FN uint8_t jmr_init_one(int i, int slice_i, int qp) {
    const int q = qp < 0 ? 0 : qp > 51 ? 51 : qp;
    const int m = slice_i ? jmr_init_I[i][0] : jmr_init_P0[i][0], n = slice_i ? jmr_init_I[i][1] : jmr_init_P0[i][1];
    int pre = ((m * q) >> 4) + n;
    pre = pre < 1 ? 1 : pre > 126 ? 126 : pre;
    return (uint8_t)(pre <= 63 ? (63 - pre) << 1 : ((pre - 64) << 1) | 1);
}
JMR_FN void jmr_init_contexts(uint8_t *st, int slice_i, int qp) {
    for (int i = 0; i < JMR_NCTX; i++) st[i] = jmr_init_one(i, slice_i, qp);
}

JMR_FN int jmr_renorm_steps(uint32_t r) { return __builtin_clz(r) - 23; }   /* r in [2, 510] */

/* Table 9-44 lookups.  A kernel may define JMR_LPS / JMR_TLPS before including this header to
   read LDS copies (a __constant__ array indexed per lane is a vector memory load, and a bin is a
   dependent chain: context -> rangeTabLPS -> context) */
#ifndef JMR_LPS
#define JMR_LPS(s, q) jmr_lps[s][q]
#define JMR_TLPS(s) jmr_trans_lps[s]
#endif

JMR_FN void jmr_bin(jmr_eng *e, int ctx, int bin) {   /* 9.3.4.2 */
    /* branch-free: both table reads depend only on the state, the outcome selects (lanes of a
       wave coding different bins stay converged) */
    const uint32_t v = e->st[ctx];
    const int s = (int)(v >> 1), mps = (int)(v & 1);
    const uint32_t lps = JMR_LPS(s, (e->range >> 6) & 3);
    const int tl = JMR_TLPS(s);
    const int lpsbin = bin != mps;
    const uint32_t r = lpsbin ? lps : e->range - lps;
    const int ns = lpsbin ? tl : (s < 62 ? s + 1 : s);
    const int nm = mps ^ (lpsbin & (s == 0));
    e->st[ctx] = (uint8_t)((ns << 1) | nm);
    const int n = jmr_renorm_steps(r);
    e->range = r << n;
    e->bits += n;
}
JMR_FN void jmr_bypass(jmr_eng *e) { e->bits++; }      /* 9.3.4.4: one step per bin       */
JMR_FN void jmr_term0(jmr_eng *e) {                    /* 9.3.4.5, binVal 0               */
    const uint32_t r = e->range - 2;
    const int n = jmr_renorm_steps(r);
    e->range = r << n;
    e->bits += n;
}
/* UEGk suffix (9.3.2.3) in bypass bins: only its length matters */
JMR_FN void jmr_eg_bypass(jmr_eng *e, unsigned v, int k) {
    for (;;) {
        if (v >= (1u << k)) { jmr_bypass(e); v -= 1u << k; k++; }
        else { e->bits += 1 + k; return; }
    }
}

/* ---- what a macroblock leaves for the context selection of its right / lower neighbours --- */
enum { JMR_K_SKIP = 0, JMR_K_INTER = 1, JMR_K_INXN = 2, JMR_K_I16 = 3 };
typedef struct jmr_mbinfo {
    uint8_t kind;         /* JMR_K_*                                                           */
    uint8_t cbp;          /* coded_block_pattern (luma | chroma << 4), 0 for P_Skip             */
    uint8_t t8;           /* transform_size_8x8_flag                                          */
    uint8_t cmode;        /* intra_chroma_pred_mode                                           */
    uint8_t cbf_dc;       /* coded_block_flag: bit 0 luma DC (I16), 1 Cb DC, 2 Cr DC            */
    uint8_t cbf_cac[2];   /* chroma AC (2x2 raster)                                           */
    uint8_t pad;
    uint16_t cbf_l;       /* luma 4x4 (raster); 8x8 transform: the 8x8 block's cbp bit on its four */
    uint16_t pad2;
    union {               /* one entropy coder per slice: the record keeps the same size for both */
        struct {
            int16_t mvd_r[4][2];  /* CABAC: mvd_l0 of the right column (rows 0..3): A of the right neighbour */
            int16_t mvd_b[4][2];  /*   of the bottom row (columns 0..3): B of the lower neighbour          */
        };
        struct {
            uint8_t tcr[8], tcb[8];   /* SymbolMode 0 (jmh_cavlc_rate.h): TotalCoeff of the right column /
                                         bottom row: luma 0..3, Cb 4..5, Cr 6..7 (zero for P_Skip)      */
        };
    };
} jmr_mbinfo;

/* a candidate of the macroblock-level RD loop (RDCost_for_macroblocks) */
typedef struct jmr_cand {
    int mb_type, cbp, i16mode, cmode, t8;
    int b8mode[4];
    const int8_t *ipm;            /* [16] 4x4 raster: -1 = predicted mode, else rem_intra_pred_mode */
    const int16_t (*mvd)[2];      /* [16] 4x4 raster: mvd_l0 of the partition covering the 4x4     */
    const int16_t (*luma)[16];    /* [16][16] as jmh_mb_result.luma                               */
    const int16_t *luma_dc;       /* [16] (I16)                                                   */
    const int16_t (*cdc)[4];      /* [2][4]                                                       */
    const int16_t (*cac)[4][16];  /* [2][4][16], [..][0] unused                                   */
    int16_t (*mvw)[2];            /* [16] work: the mvds of the partitions written so far         */
} jmr_cand;

/* the current macroblock's partial coding state inside the P8x8 RD loop (what cs_b8 carries of
   currMB: mvd, the coded_block_flag bits and the luma cbp of the decided 8x8 blocks) */
typedef struct jmr_cur {
    union {               /* one entropy coder per slice */
        struct {
            int16_t mvd[16][2];
            uint16_t cbf_l;
            uint16_t cbp;
        };
        uint8_t tc[24];   /* SymbolMode 0: the decided blocks' TotalCoeff (jmh_cavlc_rate.h)      */
    };
} jmr_cur;

/* coded_block_flag condTermFlagN (9.3.3.1.1.9) of luma 4x4 (x4, y4) of neighbour n (NULL: not
   available) for a current macroblock that is intra (cur_intra) or not */
JMR_FN int jmr_cbf_luma_term(const jmr_mbinfo *n, int cur_intra, int x4, int y4) {
    if (!n) return cur_intra;
    if (n->kind == JMR_K_SKIP) return 0;
    if (!((n->cbp >> ((y4 >> 1) * 2 + (x4 >> 1))) & 1)) return 0;
    return (n->cbf_l >> (y4 * 4 + x4)) & 1;
}

/* residual_block_cabac (7.3.5.3.3, 9.3.3.1.3): coef[0..n) in scan order, cat 0..4 (ctxBlockCat)
   or 5 (luma 8x8, no coded_block_flag: cbf_inc < 0); returns the coded_block_flag */
JMR_FN int jmr_residual(jmr_eng *e, const int16_t *coef, int n, int cat, int cbf_inc) {
    /* the significance map as a bit mask first: the bins then read no coefficient but the levels */
    uint64_t nzm = 0;
    for (int i = 0; i < n; i++)
        if (coef[i]) nzm |= (uint64_t)1 << i;
    const int last = nzm ? 63 - __builtin_clzll(nzm) : -1;
    const int cbf = last >= 0;
    if (cbf_inc >= 0) jmr_bin(e, JMR_CTX(85) + 4 * cat + cbf_inc, cbf);
    if (!cbf) return 0;
    const int so = cat == 0 ? 0 : cat == 1 ? 15 : cat == 2 ? 29 : cat == 3 ? 44 : 47;
    const int ao = cat == 0 ? 0 : cat == 1 ? 10 : cat == 2 ? 20 : cat == 3 ? 30 : 39;
    const int sig_base = cat == 5 ? JMR_CTX(402) : JMR_CTX(105) + so, last_base = cat == 5 ? JMR_CTX(417) : JMR_CTX(166) + so;
    const int abs_base = cat == 5 ? JMR_CTX(426) : JMR_CTX(227) + ao;
    for (int i = 0; i < n - 1; i++) {                 /* significance map */
        const int si = cat == 5 ? jmr_sig8x8_inc[i] : cat == 3 ? (i < 2 ? i : 2) : i;
        const int li = cat == 5 ? jmr_last8x8_inc[i] : cat == 3 ? (i < 2 ? i : 2) : i;
        const int sig = (int)((nzm >> i) & 1);
        jmr_bin(e, sig_base + si, sig);
        if (sig) {
            jmr_bin(e, last_base + li, i == last);
            if (i == last) break;
        }
    }
    int eq1 = 0, gt1 = 0;
    const int gmax = 4 - (cat == 3);
    for (uint64_t m = nzm; m;) {                      /* levels, reverse scan order */
        const int i = 63 - __builtin_clzll(m);
        m &= ~((uint64_t)1 << i);
        const int a = coef[i] < 0 ? -coef[i] : coef[i], v = a - 1;
        jmr_bin(e, abs_base + (gt1 ? 0 : (1 + eq1 < 4 ? 1 + eq1 : 4)), v > 0);
        if (v > 0) {
            const int ctx = abs_base + 5 + (gt1 < gmax ? gt1 : gmax);
            for (int k = 1; k < v && k < 14; k++) jmr_bin(e, ctx, 1);
            if (v < 14) jmr_bin(e, ctx, 0);
            else jmr_eg_bypass(e, (unsigned)(v - 14), 0);
        }
        jmr_bypass(e);                                 /* coeff_sign_flag */
        if (a == 1) eq1++;
        else gt1++;
    }
    return 1;
}

/* one mvd_l0 component (UEG3, signed, uCoff 9) with absMvdComp(A) + absMvdComp(B) = sum */
JMR_FN void jmr_mvd_comp(jmr_eng *e, int v, int sum, int comp) {
    const int base = comp ? JMR_CTX(47) : JMR_CTX(40), a = v < 0 ? -v : v;
    jmr_bin(e, base + (sum < 3 ? 0 : sum > 32 ? 2 : 1), a != 0);
    if (!a) return;
    int k = 1;
    for (; k < a && k < 9; k++) jmr_bin(e, base + (k < 4 ? k + 2 : 6), 1);
    if (a < 9) jmr_bin(e, base + (k < 4 ? k + 2 : 6), 0);
    else jmr_eg_bypass(e, (unsigned)(a - 9), 3);
    jmr_bypass(e);                                     /* sign */
}
/* the mvd of the partition whose top-left 4x4 is (x4, y4): neighbours A (x4 - 1) and B (y4 - 1)
   inside the MB from mv[] (the partitions written so far), outside from A / B */
JMR_FN void jmr_mvd(jmr_eng *e, const jmr_mbinfo *A, const jmr_mbinfo *B, const int16_t (*mv)[2], int x4, int y4, int dx,
                    int dy) {
    for (int comp = 0; comp < 2; comp++) {
        int sa = 0, sb = 0;
        if (x4 > 0) sa = mv[y4 * 4 + x4 - 1][comp];
        else if (A) sa = A->mvd_r[y4][comp];
        if (y4 > 0) sb = mv[(y4 - 1) * 4 + x4][comp];
        else if (B) sb = B->mvd_b[x4][comp];
        sa = sa < 0 ? -sa : sa;
        sb = sb < 0 ? -sb : sb;
        jmr_mvd_comp(e, comp ? dy : dx, sa + sb, comp);
    }
}
JMR_FN void jmr_put_mvd(int16_t (*mv)[2], int x4, int y4, int w4, int h4, int dx, int dy) {
    for (int y = y4; y < y4 + h4; y++)
        for (int x = x4; x < x4 + w4; x++) { mv[y * 4 + x][0] = (int16_t)dx; mv[y * 4 + x][1] = (int16_t)dy; }
}
/* sub_mb_type of P_8x8 (Table 9-38): 8x8 "1", 8x4 "00", 4x8 "011", 4x4 "010" */
JMR_FN void jmr_sub_mb_type(jmr_eng *e, int sm) {
    jmr_bin(e, JMR_CTX(21), sm == JMH_SMB8x8);
    if (sm == JMH_SMB8x8) return;
    jmr_bin(e, JMR_CTX(22), sm != JMH_SMB8x4);
    if (sm != JMH_SMB8x4) jmr_bin(e, JMR_CTX(23), sm == JMH_SMB4x8);
}
/* prev_intra4x4_pred_mode_flag / rem_intra4x4_pred_mode (FL, 3 bins) */
JMR_FN void jmr_ipred_mode(jmr_eng *e, int code) {
    jmr_bin(e, JMR_CTX(68), code < 0);
    if (code >= 0)
        for (int bit = 0; bit < 3; bit++) jmr_bin(e, JMR_CTX(69), (code >> bit) & 1);
}
/* coded_block_pattern luma bit of 8x8 block b8 (condTermFlagN: 1 when the neighbouring 8x8
   block codes no luma; internal neighbours from cbpl_cur) */
JMR_FN void jmr_cbp_bit(jmr_eng *e, const jmr_mbinfo *A, const jmr_mbinfo *B, int cbpl_cur, int b8, int bit) {
    const int bx = b8 & 1, by = b8 >> 1;
    const int ta = bx ? !((cbpl_cur >> (b8 - 1)) & 1) : (A ? !((A->cbp >> (b8 + 1)) & 1) : 0);
    const int tb = by ? !((cbpl_cur >> (b8 - 2)) & 1) : (B ? !((B->cbp >> (b8 + 2)) & 1) : 0);
    jmr_bin(e, JMR_CTX(73) + ta + 2 * tb, bit);
}

/* mb_skip_flag = 1 (a P_Skip candidate): the whole macroblock */
JMR_FN void jmr_skip(jmr_eng *e, const jmr_mbinfo *A, const jmr_mbinfo *B, jmr_mbinfo *out) {
    jmr_bin(e, JMR_CTX(11) + (A && A->kind != JMR_K_SKIP) + (B && B->kind != JMR_K_SKIP), 1);
    if (out) {
        jmr_mbinfo z = {0};
        *out = z;
    }
}

/* a whole coded macroblock (mb_skip_flag 0 in P slices, macroblock_layer; host/cabac.c
   jm_cabac_write_mb); out (may be NULL): what it leaves for its neighbours */
JMR_FN void jmr_mb(jmr_eng *e, const jmr_mbinfo *A, const jmr_mbinfo *B, const jmr_cand *r, int slice_p, int t8mode,
                   jmr_mbinfo *out) {
    const int mbt = r->mb_type;
    const int is_i8 = mbt == JMH_I8MB, is_nxn = mbt == JMH_I4MB || is_i8, is_i16 = mbt == JMH_I16MB;
    const int intra = is_nxn || is_i16, cbp = r->cbp, cbpl = cbp & 15, cbpc = cbp >> 4;
    /* the sub-macroblock types packed 4 bits each: the candidate (a private struct on the device) is
       read at constant offsets only, so it stays in registers */
    const int b8m = r->b8mode[0] | r->b8mode[1] << 4 | r->b8mode[2] << 8 | r->b8mode[3] << 12;
    jmr_mbinfo m = {0};
    m.kind = (uint8_t)(is_i16 ? JMR_K_I16 : is_nxn ? JMR_K_INXN : JMR_K_INTER);
    m.cbp = (uint8_t)cbp;
    if (slice_p) jmr_bin(e, JMR_CTX(11) + (A && A->kind != JMR_K_SKIP) + (B && B->kind != JMR_K_SKIP), 0);
    /* mb_type (9.3.2.5, Tables 9-36 / 9-37) */
    if (intra) {
        int base;
        if (slice_p) { jmr_bin(e, JMR_CTX(14), 1); base = JMR_CTX(17); }   /* prefix: intra in a P slice */
        else base = JMR_CTX(3);
        const int inc0 = slice_p ? 0 : (A && A->kind != JMR_K_INXN) + (B && B->kind != JMR_K_INXN);
        jmr_bin(e, base + inc0, is_i16);
        if (is_i16) {
            jmr_term0(e);                              /* not I_PCM */
            jmr_bin(e, base + 1 + !slice_p * 2, cbpl != 0);
            jmr_bin(e, base + 2 + !slice_p * 2, cbpc != 0);
            if (cbpc) jmr_bin(e, base + (slice_p ? 2 : 5), cbpc == 2);
            jmr_bin(e, base + (slice_p ? 3 : 6), r->i16mode >> 1);
            jmr_bin(e, base + (slice_p ? 3 : 7), r->i16mode & 1);
        }
    } else {   /* P_L0_16x16 000, P_L0_L0_16x8 011, P_L0_L0_8x16 010, P_8x8 001 */
        const int b1 = mbt == JMH_P16x8 || mbt == JMH_P8x16, b2 = mbt == JMH_P16x8 || mbt == JMH_P8x8;
        jmr_bin(e, JMR_CTX(14), 0);
        jmr_bin(e, JMR_CTX(15), b1);
        jmr_bin(e, JMR_CTX(16) + b1, b2);
    }
    if (mbt == JMH_P8x8)
        for (int i = 0; i < 4; i++) jmr_sub_mb_type(e, (b8m >> (4 * i)) & 15);
    if (is_nxn && t8mode) {
        jmr_bin(e, JMR_CTX(399) + (A && A->t8) + (B && B->t8), is_i8);
        m.t8 = (uint8_t)is_i8;
    }
    if (is_nxn)
        for (int blk = 0; blk < 16; blk += is_i8 ? 4 : 1) {
            const int x4 = ((blk >> 2) & 1) * 2 + (blk & 1), y4 = (blk >> 3) * 2 + ((blk >> 1) & 1);
            jmr_ipred_mode(e, r->ipm[y4 * 4 + x4]);
        }
    int16_t (*mv)[2] = r->mvw;                         /* mvds of the partitions written so far */
    for (int k = 0; k < 16; k++) { mv[k][0] = 0; mv[k][1] = 0; }
    if (intra) {                                       /* intra_chroma_pred_mode: TU cMax 3 */
        const int cm = r->cmode;
        const int inc = (A && (A->kind == JMR_K_INXN || A->kind == JMR_K_I16) && A->cmode) +
                        (B && (B->kind == JMR_K_INXN || B->kind == JMR_K_I16) && B->cmode);
        jmr_bin(e, JMR_CTX(64) + inc, cm > 0);
        if (cm > 0) {
            jmr_bin(e, JMR_CTX(67), cm > 1);
            if (cm > 1) jmr_bin(e, JMR_CTX(67), cm > 2);
        }
        m.cmode = (uint8_t)cm;
    } else {
        const int np = mbt == JMH_P16x16 ? 1 : mbt == JMH_P8x8 ? 4 : 2;
        for (int p = 0; p < np; p++) {
            if (mbt != JMH_P8x8) {
                const int x4 = mbt == JMH_P8x16 ? 2 * p : 0, y4 = mbt == JMH_P16x8 ? 2 * p : 0;
                const int w4 = mbt == JMH_P8x16 ? 2 : 4, h4 = mbt == JMH_P16x8 ? 2 : 4;
                const int dx = r->mvd[y4 * 4 + x4][0], dy = r->mvd[y4 * 4 + x4][1];
                jmr_mvd(e, A, B, (const int16_t(*)[2])mv, x4, y4, dx, dy);
                jmr_put_mvd(mv, x4, y4, w4, h4, dx, dy);
                continue;
            }
            const int sm = (b8m >> (4 * p)) & 15, w4 = (sm == 4 || sm == 5) ? 2 : 1, h4 = (sm == 4 || sm == 6) ? 2 : 1;
            for (int y = 0; y < 2; y += h4)
                for (int x = 0; x < 2; x += w4) {
                    const int x4 = (p & 1) * 2 + x, y4 = (p >> 1) * 2 + y;
                    const int dx = r->mvd[y4 * 4 + x4][0], dy = r->mvd[y4 * 4 + x4][1];
                    jmr_mvd(e, A, B, (const int16_t(*)[2])mv, x4, y4, dx, dy);
                    jmr_put_mvd(mv, x4, y4, w4, h4, dx, dy);
                }
        }
    }
    if (!is_i16) {                                     /* coded_block_pattern */
        for (int b8 = 0; b8 < 4; b8++) jmr_cbp_bit(e, A, B, cbpl, b8, (cbpl >> b8) & 1);
        const int ca = A ? A->cbp >> 4 : 0, cb = B ? B->cbp >> 4 : 0;
        jmr_bin(e, JMR_CTX(77) + (ca != 0) + 2 * (cb != 0), cbpc != 0);
        if (cbpc) jmr_bin(e, JMR_CTX(81) + (ca == 2) + 2 * (cb == 2), cbpc == 2);
    }
    if (!intra && cbpl && t8mode &&
        (mbt != JMH_P8x8 || b8m == 0x4444)) {
        jmr_bin(e, JMR_CTX(399) + (A && A->t8) + (B && B->t8), r->t8 != 0);
        m.t8 = (uint8_t)(r->t8 != 0);
    }
    for (int i = 0; i < 4; i++) {
        m.mvd_r[i][0] = mv[i * 4 + 3][0]; m.mvd_r[i][1] = mv[i * 4 + 3][1];
        m.mvd_b[i][0] = mv[12 + i][0]; m.mvd_b[i][1] = mv[12 + i][1];
    }
    if (cbp > 0 || is_i16) {
        jmr_bin(e, JMR_CTX(60), 0);                    /* mb_qp_delta = 0 (the previous one is 0 too) */
        if (is_i16) {                                  /* Intra16x16DCLevel */
            const int ta = A ? (A->kind == JMR_K_I16 ? A->cbf_dc & 1 : 0) : 1;
            const int tb = B ? (B->kind == JMR_K_I16 ? B->cbf_dc & 1 : 0) : 1;
            m.cbf_dc |= (uint8_t)jmr_residual(e, r->luma_dc, 16, 0, ta + 2 * tb);
        }
        for (int b8 = 0; b8 < 4; b8++) {
            if (!((cbpl >> b8) & 1)) continue;
            if (m.t8) {                                /* 8x8 block (cat 5), flag inferred 1 */
                int16_t lv[64];
                for (int j = 0; j < 4; j++) {
                    const int x4 = (b8 & 1) * 2 + (j & 1), y4 = (b8 >> 1) * 2 + (j >> 1);
                    for (int k = 0; k < 16; k++) lv[4 * k + j] = r->luma[y4 * 4 + x4][k];
                }
                jmr_residual(e, lv, 64, 5, -1);
                m.cbf_l |= (uint16_t)(0x33 << ((b8 >> 1) * 8 + (b8 & 1) * 2));
                continue;
            }
            for (int i4 = 0; i4 < 4; i4++) {
                const int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
                const int ta = x4 ? (m.cbf_l >> (y4 * 4 + x4 - 1)) & 1 : jmr_cbf_luma_term(A, intra, 3, y4);
                const int tb = y4 ? (m.cbf_l >> ((y4 - 1) * 4 + x4)) & 1 : jmr_cbf_luma_term(B, intra, x4, 3);
                const int16_t *lv = r->luma[y4 * 4 + x4];
                const int f = is_i16 ? jmr_residual(e, lv + 1, 15, 1, ta + 2 * tb) : jmr_residual(e, lv, 16, 2, ta + 2 * tb);
                m.cbf_l |= (uint16_t)(f << (y4 * 4 + x4));
            }
        }
        if (cbpc)                                      /* chroma DC (cat 3) */
            for (int uv = 0; uv < 2; uv++) {
                const int ta = A ? ((A->cbp >> 4) != 0 ? (A->cbf_dc >> (1 + uv)) & 1 : 0) : intra;
                const int tb = B ? ((B->cbp >> 4) != 0 ? (B->cbf_dc >> (1 + uv)) & 1 : 0) : intra;
                m.cbf_dc |= (uint8_t)(jmr_residual(e, r->cdc[uv], 4, 3, ta + 2 * tb) << (1 + uv));
            }
        if (cbpc == 2)                                 /* chroma AC (cat 4) */
            for (int uv = 0; uv < 2; uv++)
                for (int k = 0; k < 4; k++) {
                    const int bx = k & 1, by = k >> 1;
                    const int ta = bx ? (m.cbf_cac[uv] >> (k - 1)) & 1
                                      : A ? ((A->cbp >> 4) == 2 ? (A->cbf_cac[uv] >> (k + 1)) & 1 : 0) : intra;
                    const int tb = by ? (m.cbf_cac[uv] >> (k - 2)) & 1
                                      : B ? ((B->cbp >> 4) == 2 ? (B->cbf_cac[uv] >> (k + 2)) & 1 : 0) : intra;
                    const int f = jmr_residual(e, r->cac[uv][k] + 1, 15, 4, ta + 2 * tb);
                    m.cbf_cac[uv] |= (uint8_t)(f << k);
                }
    }
    if (out) *out = m;
}

/* RDCost_for_4x4IntraBlocks [J]: the rate of one Intra4x4 block candidate -- its pred-mode
   syntax and its luma 4x4 residual -- from the coding state at the start of the macroblock
   (JM resets the state after every candidate, so a block's current-MB neighbours carry no
   coded_block_flag bits: docs/JM_SEMANTICS.md item 55) */
JMR_FN void jmr_i4(jmr_eng *e, const jmr_mbinfo *A, const jmr_mbinfo *B, int x4, int y4, int code, const int16_t *lev) {
    jmr_ipred_mode(e, code);
    const int ta = x4 ? 0 : jmr_cbf_luma_term(A, 1, 3, y4), tb = y4 ? 0 : jmr_cbf_luma_term(B, 1, x4, 3);
    jmr_residual(e, lev, 16, 2, ta + 2 * tb);
}

/* RDCost_for_8x8IntraBlocks [J] (Transform8x8Mode): the rate of one Intra8x8 block candidate -- its
   pred-mode syntax and its luma 8x8 residual (ctxBlockCat 5, no coded_block_flag) -- from the coding
   state at the start of the macroblock (docs/JM_SEMANTICS.md item 63) */
JMR_FN void jmr_i8(jmr_eng *e, int code, const int16_t *lev64) {
    jmr_ipred_mode(e, code);
    jmr_residual(e, lev64, 64, 5, -1);
}

/* RDCost_for_8x8blocks [J] (CABAC): the rate of sub-macroblock mode sm of 8x8 block b8 --
   sub_mb_type, the mvds of its sub-partitions, its coded_block_pattern bit and, when it keeps
   coefficients (coded), the four luma 4x4 residuals -- on the running P8x8 state (cur: the
   decided 8x8 blocks), which it advances as the write would (item 56).  mvd4 / lev4: the 8x8
   block's four 4x4 in coding order (i4 = 2 * y + x) */
JMR_FN void jmr_b8(jmr_eng *e, const jmr_mbinfo *A, const jmr_mbinfo *B, jmr_cur *cur, int b8, int sm, const int16_t (*mvd4)[2],
                   int coded, const int16_t (*lev4)[16]) {
    jmr_sub_mb_type(e, sm);
    const int w4 = (sm == 4 || sm == 5) ? 2 : 1, h4 = (sm == 4 || sm == 6) ? 2 : 1;
    for (int y = 0; y < 2; y += h4)
        for (int x = 0; x < 2; x += w4) {
            const int x4 = (b8 & 1) * 2 + x, y4 = (b8 >> 1) * 2 + y;
            const int dx = mvd4[2 * y + x][0], dy = mvd4[2 * y + x][1];
            jmr_mvd(e, A, B, (const int16_t(*)[2])cur->mvd, x4, y4, dx, dy);
            jmr_put_mvd(cur->mvd, x4, y4, w4, h4, dx, dy);
        }
    jmr_cbp_bit(e, A, B, cur->cbp, b8, coded);
    if (!coded) return;
    cur->cbp |= (uint16_t)(1 << b8);
    for (int i4 = 0; i4 < 4; i4++) {
        const int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
        const int ta = x4 ? (cur->cbf_l >> (y4 * 4 + x4 - 1)) & 1 : jmr_cbf_luma_term(A, 0, 3, y4);
        const int tb = y4 ? (cur->cbf_l >> ((y4 - 1) * 4 + x4)) & 1 : jmr_cbf_luma_term(B, 0, x4, 3);
        const int f = jmr_residual(e, lev4[i4], 16, 2, ta + 2 * tb);
        cur->cbf_l |= (uint16_t)(f << (y4 * 4 + x4));
    }
}

/* the end_of_slice_flag = 0 between two macroblocks of a slice (not part of any RD rate) */
JMR_FN void jmr_end_of_mb(jmr_eng *e) { jmr_term0(e); }

#endif
