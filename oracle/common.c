/*
 * common.c — oracle tables and primitives (TEST INFRASTRUCTURE ONLY).
 *
 * Restates: JM 8.6 lencod/src/mv-search.c › Init_Motion_Search_Module (spiral tables, mvbits),
 * SATD(); image.c › UnifiedOneForthPix (quarter-pel reference) per ITU-T H.264 8.4.2.2.1;
 * block.c quant tables (quant_coef / dequant_coef, SNGL_SCAN); rdopt.c QP2QUANT;
 * QP_SCALE_CR (H.264 Table 8-15).  [J] = JM 8.6 name, unverifiable here.
 */
#include <stdlib.h>
#include "jmo_internal.h"

/* quant_coef[qp%6] (H.264 encoder scaling; JM block.c [J]); classes a=(even,even) b=(odd,odd) */
#define QROW(a, b, c) {a, c, a, c, c, b, c, b, a, c, a, c, c, b, c, b}
const int jmo_quant_coef[6][16] = {
    QROW(13107, 5243, 8066), QROW(11916, 4660, 7490), QROW(10082, 4194, 6554),
    QROW(9362, 3647, 5825),  QROW(8192, 3355, 5243),  QROW(7282, 2893, 4559)};
/* dequant_coef[qp%6] = normAdjust4x4 (H.264 8.5.9, flat scaling lists) */
const int jmo_dequant_coef[6][16] = {
    QROW(10, 16, 13), QROW(11, 18, 14), QROW(13, 20, 16),
    QROW(14, 23, 18), QROW(16, 25, 20), QROW(18, 29, 23)};
#undef QROW

/* SNGL_SCAN (4x4 frame zig-zag, H.264 Table 8-13) as raster indices */
const int jmo_scan4x4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};

/* QP2QUANT [J]: lambda for RDO-off mode decision (rdopt.c) */
const int jmo_qp2quant_tab[40] = {1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 4,
                              5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 23,
                              25, 29, 32, 36, 40, 45, 51, 57, 64, 72, 81, 91};

/* QP_SCALE_CR: QPc as a function of qPI (H.264 Table 8-15) */
const int jmo_qp_scale_cr_tab[52] = {
    0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
    18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
    34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

/* COEFF_COST [J] (block.c): cost of a |level|==1 coefficient by preceding zero run */
const int jmo_coeff_cost_tab[16] = {3, 2, 2, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

/* input->blc_size [J] (configfile.c): {width, height} for blocktype 0..7 */
const int jmo_blc_size[8][2] = {{16, 16}, {16, 16}, {16, 8}, {8, 16},
                                {8, 8},   {8, 4},   {4, 8},  {4, 4}};

int jmo_qp2quant(int qp) { return jmo_qp2quant_tab[imax(0, qp - SHIFT_QP)]; }
int jmo_qp_scale_cr(int qp) { return qp < 0 ? qp : jmo_qp_scale_cr_tab[iclip(0, 51, qp)]; }
int jmo_qpc(int qpi, int qpbd) { qpi = iclip(-qpbd, 51, qpi); return qpi < 0 ? qpi : jmo_qp_scale_cr_tab[qpi]; }

/* mvbits[v] [J] (Init_Motion_Search_Module): length of se(v) Exp-Golomb code, 9.1 */
int jmo_mvbits(int v) {
    if (v == 0) return 1;
    unsigned a = (unsigned)iabs(v);
    int lg = 31 - __builtin_clz(a);          /* floor(log2|v|) */
    return 2 * lg + 3;
}

/* Init_Motion_Search_Module spiral [J]: entry 0 = (0,0); ring l: (i,-l),(i,l) for
 * i in [-l+1,l-1], then (-l,i),(l,i) for i in [-l,l]. */
void jmo_spiral(int range, int32_t *sx, int32_t *sy) {
    int k = 1;
    sx[0] = sy[0] = 0;
    for (int l = 1; l <= range; l++) {
        for (int i = -l + 1; i < l; i++) {
            sx[k] = i; sy[k] = -l; k++;
            sx[k] = i; sy[k] = l;  k++;
        }
        for (int i = -l; i <= l; i++) {
            sx[k] = -l; sy[k] = i; k++;
            sx[k] = l;  sy[k] = i; k++;
        }
    }
}

void jmo_init_spiral(jmo_ctx *c) {
    int n = c->npos, side = 2 * c->sr + 1;
    c->spiral_x = (int32_t *)malloc(sizeof(int32_t) * n);
    c->spiral_y = (int32_t *)malloc(sizeof(int32_t) * n);
    c->spiral_of = (int32_t *)malloc(sizeof(int32_t) * n);
    jmo_spiral(c->sr, c->spiral_x, c->spiral_y);
    for (int k = 0; k < n; k++)
        c->spiral_of[(c->spiral_y[k] + c->sr) * side + (c->spiral_x[k] + c->sr)] = k;
}

/* ---- luma quarter-pel interpolation, H.264 8.4.2.2.1 (normative) ----------------------- */
static inline int tap6(int a, int b, int c, int d, int e, int f) {
    return a - 5 * b + 20 * c + 20 * d - 5 * e + f;
}
/* one sample at quarter-pel (X, Y) from integer samples PX(x, y) (clamped access), Clip1 = maxv */
#define QPEL_BODY(PX)                                                                                   \
    int x = X >> 2, y = Y >> 2, fx = X & 3, fy = Y & 3;                                                  \
    int G = PX(x, y);                                                                                   \
    if (fx == 0 && fy == 0) return G;                                                                   \
    /* b1 / h1: horizontal / vertical half-pel intermediates between (x,y) and (x+1,y) / (x,y+1) */      \
    int b = clipv(maxv, (HB1(PX, x, y) + 16) >> 5);                                                     \
    int hh = clipv(maxv, (VH1(PX, x, y) + 16) >> 5);                                                    \
    int jj = 0;                                                                                         \
    if ((fx == 2 && fy != 0) || (fy == 2 && fx != 0)) {                                                 \
        int j1 = tap6(VH1(PX, x - 2, y), VH1(PX, x - 1, y), VH1(PX, x, y), VH1(PX, x + 1, y),          \
                      VH1(PX, x + 2, y), VH1(PX, x + 3, y));                                            \
        jj = clipv(maxv, (j1 + 512) >> 10);                                                            \
    }                                                                                                   \
    int s_ = clipv(maxv, (HB1(PX, x, y + 1) + 16) >> 5);   /* b at row y+1   */                         \
    int m = clipv(maxv, (VH1(PX, x + 1, y) + 16) >> 5);    /* h at column x+1 */                        \
    int H_ = PX(x + 1, y), M = PX(x, y + 1);                                                             \
    switch (fy * 4 + fx) {                                                                              \
    case 1: return (G + b + 1) >> 1;        /* a */                                                     \
    case 2: return b;                       /* b */                                                     \
    case 3: return (H_ + b + 1) >> 1;       /* c */                                                     \
    case 4: return (G + hh + 1) >> 1;       /* d */                                                     \
    case 5: return (b + hh + 1) >> 1;       /* e */                                                     \
    case 6: return (b + jj + 1) >> 1;       /* f */                                                     \
    case 7: return (b + m + 1) >> 1;        /* g */                                                     \
    case 8: return hh;                      /* h */                                                     \
    case 9: return (hh + jj + 1) >> 1;      /* i */                                                     \
    case 10: return jj;                     /* j */                                                     \
    case 11: return (jj + m + 1) >> 1;      /* k */                                                     \
    case 12: return (M + hh + 1) >> 1;      /* n */                                                     \
    case 13: return (hh + s_ + 1) >> 1;     /* p */                                                     \
    case 14: return (jj + s_ + 1) >> 1;     /* q */                                                     \
    case 15: return (m + s_ + 1) >> 1;      /* r */                                                     \
    }                                                                                                   \
    return G;
#define HB1(PX, xx, yy) tap6(PX((xx) - 2, yy), PX((xx) - 1, yy), PX(xx, yy), PX((xx) + 1, yy), PX((xx) + 2, yy), PX((xx) + 3, yy))
#define VH1(PX, xx, yy) tap6(PX(xx, (yy) - 2), PX(xx, (yy) - 1), PX(xx, yy), PX(xx, (yy) + 1), PX(xx, (yy) + 2), PX(xx, (yy) + 3))
#define PX8(xx, yy) p[iclip(0, h - 1, yy) * s + iclip(0, w - 1, xx)]
int jmo_luma_qpel_sample(const uint8_t *p, int w, int h, int s, int X, int Y) {
    const int maxv = 255;
    QPEL_BODY(PX8)
}
int jmo_qpel_px(const pel *p, int w, int h, int s, int X, int Y, int maxv) {
    QPEL_BODY(PX8)
}
#undef PX8
#undef HB1
#undef VH1
#undef QPEL_BODY

/* UnifiedOneForthPix [J]: 16 phase planes of the reference, padded by JMO_PAD so that
 * clamping the integer position into [-PAD, W-1+PAD] (keeping the phase) equals the
 * spec's per-tap coordinate clamping (PAD >= 3). */
void jmo_build_qpel(jmo_ctx *c) {
    int P = JMO_PAD, qs = c->qstride, qh = c->H + 2 * P;
    for (int ph = 0; ph < 16; ph++) {
        int fx = ph & 3, fy = ph >> 2;
        pel *pl = c->qpel + (size_t)ph * c->qplane;
        for (int y = 0; y < qh; y++)
            for (int x = 0; x < qs; x++)
                pl[y * qs + x] = (pel)jmo_qpel_px(c->refY, c->W, c->H, c->W, 4 * (x - P) + fx, 4 * (y - P) + fy, c->maxv);
    }
}

int jmo_qpel_at(const jmo_ctx *c, int X, int Y) {
    int P = JMO_PAD;
    int x = iclip(-P, c->W - 1 + P, X >> 2), y = iclip(-P, c->H - 1 + P, Y >> 2);
    int ph = (Y & 3) * 4 + (X & 3);
    return c->qpel[(size_t)ph * c->qplane + (size_t)(y + P) * c->qstride + (x + P)];
}

/* SATD() [J] (mv-search.c): 4x4 Hadamard, sum |.|, >>1  (the sum is always even, so this
 * equals JM>=10's (sum+1)>>1);  plain SAD when use_hadamard == 0. d[] raster. */
int jmo_satd_block(const int32_t d[16], int use_hadamard) {
    int satd = 0;
    if (!use_hadamard) {
        for (int k = 0; k < 16; k++) satd += iabs(d[k]);
        return satd;
    }
    int m[16], t[16];
    for (int x = 0; x < 4; x++) {        /* vertical (columns) */
        int a0 = d[x] + d[12 + x], a1 = d[4 + x] + d[8 + x];
        int a2 = d[4 + x] - d[8 + x], a3 = d[x] - d[12 + x];
        m[x] = a0 + a1; m[8 + x] = a0 - a1; m[4 + x] = a2 + a3; m[12 + x] = a3 - a2;
    }
    for (int y = 0; y < 4; y++) {        /* horizontal (rows) */
        int *r = m + 4 * y;
        int a0 = r[0] + r[3], a1 = r[1] + r[2], a2 = r[1] - r[2], a3 = r[0] - r[3];
        t[4 * y + 0] = a0 + a1; t[4 * y + 2] = a0 - a1;
        t[4 * y + 1] = a2 + a3; t[4 * y + 3] = a3 - a2;
    }
    for (int k = 0; k < 16; k++) satd += iabs(t[k]);
    return satd >> 1;
}
int jmo_satd4x4(const int32_t *diff, int use_hadamard) { return jmo_satd_block(diff, use_hadamard); }

/* forward 4x4 core transform (encoder; block.c dct_luma [J]) raster in place */
void jmo_fwd4x4(int32_t m[16]) {
    for (int y = 0; y < 4; y++) {        /* horizontal */
        int32_t *r = m + 4 * y;
        int p0 = r[0] + r[3], p3 = r[0] - r[3], p1 = r[1] + r[2], p2 = r[1] - r[2];
        r[0] = p0 + p1; r[2] = p0 - p1; r[1] = 2 * p3 + p2; r[3] = p3 - 2 * p2;
    }
    for (int x = 0; x < 4; x++) {        /* vertical */
        int p0 = m[x] + m[12 + x], p3 = m[x] - m[12 + x];
        int p1 = m[4 + x] + m[8 + x], p2 = m[4 + x] - m[8 + x];
        m[x] = p0 + p1; m[8 + x] = p0 - p1; m[4 + x] = 2 * p3 + p2; m[12 + x] = p3 - 2 * p2;
    }
}
void jmo_forward4x4(const int32_t *in, int32_t *out) {
    memcpy(out, in, 16 * sizeof(int32_t));
    jmo_fwd4x4(out);
}

/* inverse 4x4 (H.264 8.5.12.2): rows first, then columns; no final shift */
static void inv4x4_core(const int32_t in[16], int32_t out[16]) {
    int32_t t[16];
    for (int y = 0; y < 4; y++) {
        const int32_t *d = in + 4 * y;
        int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
        t[4 * y + 0] = e0 + e3; t[4 * y + 1] = e1 + e2; t[4 * y + 2] = e1 - e2; t[4 * y + 3] = e0 - e3;
    }
    for (int x = 0; x < 4; x++) {
        int d0 = t[x], d1 = t[4 + x], d2 = t[8 + x], d3 = t[12 + x];
        int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
        out[x] = e0 + e3; out[4 + x] = e1 + e2; out[8 + x] = e1 - e2; out[12 + x] = e0 - e3;
    }
}
void jmo_inverse4x4(const int32_t *in, int32_t *out) { inv4x4_core(in, out); }

/* inverse transform + reconstruction: clip((r + (pred<<6) + 32) >> 6) */
void jmo_inv4x4_add(const int32_t m[16], const pel *pred, int pstride, pel *out, int ostride, int maxv) {
    int32_t r[16];
    inv4x4_core(m, r);
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++)
            out[y * ostride + x] = (pel)clipv(maxv, (r[4 * y + x] + (pred[y * pstride + x] << DQ_BITS) + DQ_ROUND) >> DQ_BITS);
}

/* ======================================================================================== */
/*  8x8 transform (High profile, Transform8x8Mode) — JM FRExt block.c › dct_luma8x8 [J]      */
/* ======================================================================================== */
/* normAdjust8x8 position class (H.264 8.5.9): 0 (i%4==0,j%4==0), 1 (odd,odd), 2 (2 mod 4 both),
 * 3 (0 mod 4 / odd), 4 (0 mod 4 / 2 mod 4), 5 otherwise */
int jmo_class8(int x, int y) {
    if (!(x & 3) && !(y & 3)) return 0;
    if ((x & 1) && (y & 1)) return 1;
    if ((x & 3) == 2 && (y & 3) == 2) return 2;
    if ((!(x & 3) && (y & 1)) || ((x & 1) && !(y & 3))) return 3;
    if ((!(x & 3) && (y & 3) == 2) || ((x & 3) == 2 && !(y & 3))) return 4;
    return 5;
}
/* dequant_coef8 = normAdjust8x8 v[m][class] (H.264 Table 8-16 / 8.5.9) */
const int jmo_dequant8_cls[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26},
                                    {26, 23, 42, 24, 33, 31}, {28, 25, 45, 26, 35, 33},
                                    {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};
/* quant_coef8 [J] by class: q * v == 2^18 * (4x4 class norm), rounded as in JM's table */
const int jmo_quant8_cls[6][6] = {{13107, 11428, 20972, 12222, 16777, 15481},
                                  {11916, 10826, 19174, 11058, 14980, 14290},
                                  {10082, 8943, 15978, 9675, 12710, 11985},
                                  {9362, 8228, 14913, 8931, 11984, 11259},
                                  {8192, 7346, 13159, 7740, 10486, 9777},
                                  {7282, 6428, 11570, 6830, 9118, 8640}};
/* COEFF_COST8x8[0] [J]: cost of a |level|==1 coefficient by preceding zero run (64-scan) */
int jmo_coeff_cost8(int run) { return run < 4 ? 3 : run < 12 ? 2 : run < 24 ? 1 : 0; }

/* SNGL_SCAN8x8 (8x8 frame zig-zag, H.264 Table 8-13... same order as JPEG): raster index */
void jmo_scan8x8(int scan[64]) {
    int k = 0;
    for (int s = 0; s < 15; s++) {
        if (s & 1) for (int x = s < 8 ? s : 7; x >= 0 && s - x < 8; x--) scan[k++] = (s - x) * 8 + x;
        else for (int x = s < 8 ? 0 : s - 7; x <= 7 && s - x >= 0; x++) scan[k++] = (s - x) * 8 + x;
    }
}

/* one 8-point forward butterfly (JM forward8x8 [J]) */
static void fwd8(const int32_t *in, int st, int32_t *out, int ost) {
    int x0 = in[0], x1 = in[st], x2 = in[2 * st], x3 = in[3 * st], x4 = in[4 * st], x5 = in[5 * st],
        x6 = in[6 * st], x7 = in[7 * st];
    int a0 = x0 + x7, a1 = x1 + x6, a2 = x2 + x5, a3 = x3 + x4;
    int b0 = a0 + a3, b1 = a1 + a2, b2 = a0 - a3, b3 = a1 - a2;
    int a4 = x0 - x7, a5 = x1 - x6, a6 = x2 - x5, a7 = x3 - x4;
    int b4 = a5 + a6 + ((a4 >> 1) + a4), b5 = a4 - a7 - ((a6 >> 1) + a6);
    int b6 = a4 + a7 - ((a5 >> 1) + a5), b7 = a5 - a6 + ((a7 >> 1) + a7);
    out[0] = b0 + b1; out[ost] = b4 + (b7 >> 2); out[2 * ost] = b2 + (b3 >> 1); out[3 * ost] = b5 + (b6 >> 2);
    out[4 * ost] = b0 - b1; out[5 * ost] = b6 - (b5 >> 2); out[6 * ost] = (b2 >> 1) - b3; out[7 * ost] = (b4 >> 2) - b7;
}
void jmo_fwd8x8(int32_t m[64]) {          /* raster in place: rows, then columns */
    int32_t t[64];
    for (int y = 0; y < 8; y++) fwd8(m + 8 * y, 1, t + 8 * y, 1);
    for (int x = 0; x < 8; x++) fwd8(t + x, 8, m + x, 8);
}
/* one 8-point inverse (H.264 8.5.13.2) */
static void inv8(const int32_t *in, int st, int32_t *out, int ost) {
    int d0 = in[0], d1 = in[st], d2 = in[2 * st], d3 = in[3 * st], d4 = in[4 * st], d5 = in[5 * st],
        d6 = in[6 * st], d7 = in[7 * st];
    int a0 = d0 + d4, a4 = d0 - d4, a2 = (d2 >> 1) - d6, a6 = d2 + (d6 >> 1);
    int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
    int a1 = -d3 + d5 - d7 - (d7 >> 1), a3 = d1 + d7 - d3 - (d3 >> 1);
    int a5 = -d1 + d7 + d5 + (d5 >> 1), a7 = d3 + d5 + d1 + (d1 >> 1);
    int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
    out[0] = b0 + b7; out[ost] = b2 + b5; out[2 * ost] = b4 + b3; out[3 * ost] = b6 + b1;
    out[4 * ost] = b6 - b1; out[5 * ost] = b4 - b3; out[6 * ost] = b2 - b5; out[7 * ost] = b0 - b7;
}
void jmo_inverse8x8(const int32_t *in, int32_t *out) {   /* rows first, then columns */
    int32_t t[64];
    for (int y = 0; y < 8; y++) inv8(in + 8 * y, 1, t + 8 * y, 1);
    for (int x = 0; x < 8; x++) inv8(t + x, 8, out + x, 8);
}
void jmo_inv8x8_add(const int32_t m[64], const pel *pred, int pstride, pel *out, int ostride, int maxv) {
    int32_t r[64];
    jmo_inverse8x8(m, r);
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++)
            out[y * ostride + x] = (pel)clipv(maxv, (r[8 * y + x] + (pred[y * pstride + x] << DQ_BITS) + DQ_ROUND) >> DQ_BITS);
}
/* HadamardSAD8x8 [J]: (sum |H8 D H8| + 2) >> 2; SAD when use_hadamard == 0.  d[] raster. */
int jmo_satd8x8(const int32_t d[64], int use_hadamard) {
    int sum = 0;
    if (!use_hadamard) {
        for (int k = 0; k < 64; k++) sum += iabs(d[k]);
        return sum;
    }
    int32_t m[64];
    memcpy(m, d, sizeof(m));
    for (int pass = 0; pass < 2; pass++)
        for (int i = 0; i < 8; i++) {
            int st = pass ? 8 : 1;
            int32_t *v = pass ? m + i : m + 8 * i;
            for (int h = 1; h < 8; h <<= 1)
                for (int k = 0; k < 8; k++)
                    if (!(k & h)) { int a = v[k * st], b = v[(k + h) * st]; v[k * st] = a + b; v[(k + h) * st] = a - b; }
        }
    for (int k = 0; k < 64; k++) sum += iabs(m[k]);
    return (sum + 2) >> 2;
}
