/*
 * decoder.c — minimal normative H.264 decoder for closed-loop checks (TEST INFRASTRUCTURE ONLY).
 *
 * Scope: the Baseline / High subset the host encoder emits — progressive frames, 4:2:0 8-bit,
 * one or more slices per picture (raster order, no ASO), CAVLC, I and P slices, one reference picture, no FMO/ASO/redundant
 * slices, POC type 0; High: transform_size_8x8_flag (8x8 residual, Intra_8x8), flat scaling.  Written from ITU-T H.264 clauses 7.3 (syntax), 8.3 (intra), 8.4
 * (inter, MVP via "partition already decoded" tracking, independent of the encoder's JM
 * shape rules), 8.5 (scaling/inverse transforms), 8.7 (deblocking), 9.1/9.2 (Exp-Golomb,
 * CAVLC).  This is SURVEY.md §2 row 20: JM's ldecod closed-loop role — an encoder is correct
 * iff decoder output == encoder recon.
 */
#include <stdio.h>
#include <stdlib.h>
#include "jmo_internal.h"

/* ---- RBSP bit reader -------------------------------------------------------------------- */
typedef struct { const uint8_t *p; long n, pos; int err; } br_t;
static int rb(br_t *b) {
    if (b->pos >= b->n * 8) { b->err = 1; return 0; }
    int v = (b->p[b->pos >> 3] >> (7 - (b->pos & 7))) & 1;
    b->pos++;
    return v;
}
static uint32_t rbits(br_t *b, int n) { uint32_t v = 0; while (n--) v = (v << 1) | rb(b); return v; }
static uint32_t peek(br_t *b, int n) { long s = b->pos; int e = b->err; uint32_t v = rbits(b, n); b->pos = s; b->err = e; return v; }
static uint32_t rue(br_t *b) {
    int z = 0;
    while (!rb(b)) { if (++z > 31 || b->err) { b->err = 1; return 0; } }
    return (1u << z) - 1 + rbits(b, z);
}
static int32_t rse(br_t *b) { uint32_t k = rue(b); return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2); }

/* ---- CAVLC tables (same normative tables, decoded by prefix match) -------------------- */
static const uint8_t ct_len[3][4][17] = {
    {{1, 6, 8, 9, 10, 11, 13, 13, 13, 14, 14, 15, 15, 16, 16, 16, 16}, {0, 2, 6, 8, 9, 10, 11, 13, 13, 14, 14, 15, 15, 15, 16, 16, 16},
     {0, 0, 3, 7, 8, 9, 10, 11, 13, 13, 14, 14, 15, 15, 16, 16, 16}, {0, 0, 0, 5, 6, 7, 8, 9, 10, 11, 13, 14, 14, 15, 15, 16, 16}},
    {{2, 6, 6, 7, 8, 8, 9, 11, 11, 12, 12, 12, 13, 13, 13, 14, 14}, {0, 2, 5, 6, 6, 7, 8, 9, 11, 11, 12, 12, 13, 13, 14, 14, 14},
     {0, 0, 3, 6, 6, 7, 8, 9, 11, 11, 12, 12, 13, 13, 13, 14, 14}, {0, 0, 0, 4, 4, 5, 6, 6, 7, 9, 11, 11, 12, 13, 13, 13, 14}},
    {{4, 6, 6, 6, 7, 7, 7, 7, 8, 8, 9, 9, 9, 10, 10, 10, 10}, {0, 4, 5, 5, 5, 5, 6, 6, 7, 8, 8, 9, 9, 9, 10, 10, 10},
     {0, 0, 4, 5, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 10}, {0, 0, 0, 4, 4, 4, 4, 4, 5, 6, 7, 8, 8, 9, 10, 10, 10}}};
static const uint8_t ct_code[3][4][17] = {
    {{1, 5, 7, 7, 7, 7, 15, 11, 8, 15, 11, 15, 11, 15, 11, 7, 4}, {0, 1, 4, 6, 6, 6, 6, 14, 10, 14, 10, 14, 10, 1, 14, 10, 6},
     {0, 0, 1, 5, 5, 5, 5, 5, 13, 9, 13, 9, 13, 9, 13, 9, 5}, {0, 0, 0, 3, 3, 4, 4, 4, 4, 4, 12, 12, 8, 12, 8, 12, 8}},
    {{3, 11, 7, 7, 7, 4, 7, 15, 11, 15, 11, 8, 15, 11, 7, 9, 7}, {0, 2, 7, 10, 6, 6, 6, 6, 14, 10, 14, 10, 14, 10, 11, 8, 6},
     {0, 0, 3, 9, 5, 5, 5, 5, 13, 9, 13, 9, 13, 9, 6, 10, 5}, {0, 0, 0, 5, 4, 6, 8, 4, 4, 4, 12, 8, 12, 12, 8, 1, 4}},
    {{15, 15, 11, 8, 15, 11, 9, 8, 15, 11, 15, 11, 8, 13, 9, 5, 1}, {0, 14, 15, 12, 10, 8, 14, 10, 14, 14, 10, 14, 10, 7, 12, 8, 4},
     {0, 0, 13, 14, 11, 9, 13, 9, 13, 10, 13, 9, 13, 9, 11, 7, 3}, {0, 0, 0, 12, 11, 10, 9, 8, 13, 12, 12, 12, 8, 12, 10, 6, 2}}};
static const uint8_t ctdc_len[4][5] = {{2, 6, 6, 6, 6}, {0, 1, 6, 7, 8}, {0, 0, 3, 7, 8}, {0, 0, 0, 6, 7}};
static const uint8_t ctdc_code[4][5] = {{1, 7, 4, 3, 2}, {0, 1, 6, 3, 3}, {0, 0, 1, 2, 2}, {0, 0, 0, 5, 0}};
static const uint8_t tz_len[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6}, {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},
    {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5}, {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5}, {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6}, {6, 4, 5, 3, 2, 2, 3, 3, 6}, {6, 6, 4, 2, 2, 3, 2, 5}, {5, 5, 3, 2, 2, 2, 4}, {4, 4, 3, 3, 1, 3},
    {4, 4, 2, 1, 3}, {3, 3, 1, 2}, {2, 2, 1}, {1, 1}};
static const uint8_t tz_code[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0}, {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},
    {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0}, {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0}, {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0}, {1, 1, 1, 3, 3, 2, 2, 1, 0}, {1, 0, 1, 3, 2, 1, 1, 1}, {1, 0, 1, 3, 2, 1, 1}, {0, 1, 1, 2, 1, 3},
    {0, 1, 1, 1, 1}, {0, 1, 1, 1}, {0, 1, 1}, {0, 1}};
static const uint8_t tzdc_len[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
static const uint8_t tzdc_code[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
static const uint8_t rb_len[7][15] = {{1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3}, {2, 3, 3, 3, 3, 3, 3},
                                      {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
static const uint8_t rb_code[7][15] = {{1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0}, {3, 0, 1, 3, 2, 5, 4},
                                       {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}};
/* Table 9-4: codeNum -> coded_block_pattern (ChromaArrayType 1) */
static const uint8_t cbp_intra[48] = {47, 31, 15, 0, 23, 27, 29, 30, 7, 11, 13, 14, 39, 43, 45, 46, 16, 3, 5, 10, 12, 19, 21, 26,
                                      28, 35, 37, 42, 44, 1, 2, 4, 8, 17, 18, 20, 24, 6, 9, 22, 25, 32, 33, 34, 36, 40, 38, 41};
static const uint8_t cbp_inter[48] = {0, 16, 1, 2, 4, 8, 32, 3, 5, 10, 12, 15, 47, 7, 11, 13, 14, 6, 9, 31, 35, 37, 42, 44,
                                      33, 34, 36, 40, 39, 43, 45, 46, 17, 18, 20, 24, 19, 21, 26, 28, 23, 27, 29, 30, 22, 25, 38, 41};

static int match(br_t *b, int code, int len) {
    if (len <= 0) return 0;
    if ((int)peek(b, len) == code) { b->pos += len; return 1; }
    return 0;
}

/* residual_block_cavlc: fills coeffLevel[0..maxn) (scan order); returns TotalCoeff or -1 */
static int read_block(br_t *b, int nC, int maxn, int *coef) {
    for (int i = 0; i < maxn; i++) coef[i] = 0;
    int tc = -1, t1 = -1;
    if (nC == -1) {
        for (int a = 0; a < 4 && tc < 0; a++)
            for (int c = a; c < 5; c++) if (match(b, ctdc_code[a][c], ctdc_len[a][c])) { t1 = a; tc = c; break; }
    } else if (nC >= 8) {
        int v = rbits(b, 6);
        if (v == 3) { tc = 0; t1 = 0; } else { tc = (v >> 2) + 1; t1 = v & 3; }
    } else {
        int t = nC < 2 ? 0 : nC < 4 ? 1 : 2;
        for (int a = 0; a < 4 && tc < 0; a++)
            for (int c = a; c < 17; c++) if (c > 0 || a == 0) if (match(b, ct_code[t][a][c], ct_len[t][a][c])) { t1 = a; tc = c; break; }
    }
    if (tc < 0 || tc > maxn || t1 > tc) return -1;
    if (!tc) return 0;
    int lev[16];
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = 0; i < tc; i++) {
        if (i < t1) { lev[i] = rb(b) ? -1 : 1; continue; }
        int prefix = 0;
        while (!rb(b)) { if (++prefix > 15 || b->err) return -1; }
        int size = (prefix == 14 && sl == 0) ? 4 : (prefix >= 15 ? prefix - 3 : sl);
        int code = (imin(15, prefix) << sl) + (size ? (int)rbits(b, size) : 0);
        if (prefix >= 15 && sl == 0) code += 15;
        if (i == t1 && t1 < 3) code += 2;
        lev[i] = (code & 1) ? (-code - 1) >> 1 : (code + 2) >> 1;
        if (sl == 0) sl = 1;
        if (iabs(lev[i]) > (3 << (sl - 1)) && sl < 6) sl++;
    }
    int tz = 0;
    if (tc < maxn) {
        tz = -1;
        if (nC == -1) { for (int z = 0; z <= 4 - tc; z++) if (match(b, tzdc_code[tc - 1][z], tzdc_len[tc - 1][z])) { tz = z; break; } }
        else { for (int z = 0; z <= 16 - tc; z++) if (match(b, tz_code[tc - 1][z], tz_len[tc - 1][z])) { tz = z; break; } }
        if (tz < 0) return -1;
    }
    int zl = tz, run[16];
    for (int i = 0; i < tc - 1; i++) {
        run[i] = 0;
        if (zl > 0) {
            int t = zl > 6 ? 6 : zl - 1, got = -1;
            for (int r = 0; r <= imin(zl, 14); r++) if (match(b, rb_code[t][r], rb_len[t][r])) { got = r; break; }
            if (got < 0) return -1;
            run[i] = got;
        }
        zl -= run[i];
    }
    run[tc - 1] = zl;
    int pos = -1;
    for (int i = tc - 1; i >= 0; i--) {
        pos += run[i] + 1;
        if (pos >= maxn) return -1;
        coef[pos] = lev[i];
    }
    return tc;
}

/* ---- decoder state -------------------------------------------------------------------- */
typedef struct {
    int mbtype;           /* 0 P_L0 inter, 1 I4x4, 2 I16, 3 P_Skip, 4 I8x8 */
    int t8;               /* transform_size_8x8_flag */
    int intra;
    int qp;
    uint8_t tc[24];       /* total_coeff: 16 luma (raster 4x4), 4 cb, 4 cr               */
    int nzblk;            /* luma 4x4 blocks with non-zero coefficients (bit raster)      */
    int8_t ipm[16];
} mbinfo;

struct jmo_dec {
    char err[256];
    int have_sps, have_pps;
    int mbw, mbh, W, H, crop_l, crop_r, crop_t, crop_b;
    int log2_fn, poc_type, log2_poc;
    int num_ref_l0, init_qp, cqp_off, dfc_present, cip, t8mode;
    uint8_t *cur[3], *ref[3];
    int have_ref;
    mbinfo *mi;
    int16_t *mv;          /* per 4x4 [2] */
    int8_t *refi;         /* per 4x4 */
    int8_t *dec4;         /* per 4x4: decoded in the current picture */
    int dis_dbf, offA, offB;
    int slice_first;      /* first MB of the current slice: MBs before it are unavailable (6.4.8) */
    int mbs_done;         /* MBs of the current picture decoded so far (a picture may have many slices) */
};

int jmo_dec_create(jmo_dec **out) { *out = (jmo_dec *)calloc(1, sizeof(jmo_dec)); return *out ? 0 : JMH_E_OOM; }
void jmo_dec_destroy(jmo_dec *d) {
    if (!d) return;
    for (int i = 0; i < 3; i++) { free(d->cur[i]); free(d->ref[i]); }
    free(d->mi); free(d->mv); free(d->refi); free(d->dec4);
    free(d);
}
const char *jmo_dec_error(const jmo_dec *d) { return d->err; }

static void alloc_pics(jmo_dec *d) {
    for (int i = 0; i < 3; i++) { free(d->cur[i]); free(d->ref[i]); }
    size_t ls = (size_t)d->W * d->H;
    d->cur[0] = calloc(ls, 1); d->cur[1] = calloc(ls / 4, 1); d->cur[2] = calloc(ls / 4, 1);
    d->ref[0] = calloc(ls, 1); d->ref[1] = calloc(ls / 4, 1); d->ref[2] = calloc(ls / 4, 1);
    free(d->mi); free(d->mv); free(d->refi); free(d->dec4);
    d->mi = calloc((size_t)d->mbw * d->mbh, sizeof(mbinfo));
    d->mv = calloc(ls / 16 * 2, sizeof(int16_t));
    d->refi = calloc(ls / 16, 1);
    d->dec4 = calloc(ls / 16, 1);
    d->have_ref = 0;
}

static int parse_sps(jmo_dec *d, br_t *b) {
    int profile = rbits(b, 8);
    rbits(b, 16);
    rue(b);
    if (profile == 100) {                 /* High: only 4:2:0 8-bit with flat scaling lists */
        if (rue(b) != 1 || rue(b) != 0 || rue(b) != 0 || rb(b) || rb(b)) {
            snprintf(d->err, sizeof d->err, "High profile SPS options unsupported");
            return -1;
        }
    } else if (profile >= 100) { snprintf(d->err, sizeof d->err, "profile %d unsupported", profile); return -1; }
    d->log2_fn = rue(b) + 4;
    d->poc_type = rue(b);
    if (d->poc_type != 0) { snprintf(d->err, sizeof d->err, "poc type"); return -1; }
    d->log2_poc = rue(b) + 4;
    rue(b);                       /* num_ref_frames */
    rb(b);
    d->mbw = rue(b) + 1; d->mbh = rue(b) + 1;
    if (!rb(b)) { snprintf(d->err, sizeof d->err, "field coding unsupported"); return -1; }
    rb(b);
    d->crop_l = d->crop_r = d->crop_t = d->crop_b = 0;
    if (rb(b)) { d->crop_l = rue(b); d->crop_r = rue(b); d->crop_t = rue(b); d->crop_b = rue(b); }
    rb(b);                        /* vui */
    d->W = 16 * d->mbw; d->H = 16 * d->mbh;
    alloc_pics(d);
    d->have_sps = 1;
    return b->err ? -1 : 0;
}
static int parse_pps(jmo_dec *d, br_t *b) {
    rue(b); rue(b);
    if (rb(b)) { snprintf(d->err, sizeof d->err, "CABAC unsupported"); return -1; }
    rb(b);
    if (rue(b)) { snprintf(d->err, sizeof d->err, "FMO unsupported"); return -1; }
    d->num_ref_l0 = rue(b) + 1;
    rue(b);
    if (rb(b) || rbits(b, 2)) { snprintf(d->err, sizeof d->err, "weighted prediction unsupported"); return -1; }
    d->init_qp = 26 + rse(b);
    rse(b);
    d->cqp_off = rse(b);
    d->dfc_present = rb(b);
    d->cip = rb(b);
    rb(b);
    d->t8mode = 0;
    /* more_rbsp_data(): anything before the rbsp_stop_one_bit */
    long last = b->n * 8 - 1;
    while (last >= 0 && !((b->p[last >> 3] >> (7 - (last & 7))) & 1)) last--;
    if (b->pos < last) {
        d->t8mode = rb(b);
        if (rb(b)) { snprintf(d->err, sizeof d->err, "scaling matrices unsupported"); return -1; }
        if (rse(b) != d->cqp_off) { snprintf(d->err, sizeof d->err, "second_chroma_qp_index_offset unsupported"); return -1; }
    }
    d->have_pps = 1;
    return b->err ? -1 : 0;
}

/* ---- intra prediction (8.3) ------------------------------------------------------------ */
static int avail_mb(const jmo_dec *d, int mx, int my, int cmx, int cmy) {
    if (mx < 0 || my < 0 || mx >= d->mbw || my >= d->mbh || my * d->mbw + mx < d->slice_first) return 0;
    return my < cmy || (my == cmy && mx < cmx);
}
/* availability of luma sample at MB-relative (x,y) for intra 4x4 block at (bx,by) */
static int lavail(const jmo_dec *d, int mx, int my, int x, int y, int blk_idx) {
    if (x > 15 || y > 15) { if (x > 15 && y < 0) return avail_mb(d, mx + 1, my - 1, mx, my); return 0; }
    if (x < 0 && y < 0) return avail_mb(d, mx - 1, my - 1, mx, my);
    if (x < 0) return avail_mb(d, mx - 1, my, mx, my);
    if (y < 0) return avail_mb(d, mx, my - 1, mx, my);
    (void)blk_idx;
    return 1;
}
static void pred4x4(const jmo_dec *d, int mx, int my, int bx, int by, int blk_idx, int mode, uint8_t *pr, int *ok) {
    const uint8_t *R = d->cur[0];
    int W = d->W, X = 16 * mx + bx, Y = 16 * my + by;
    int up = lavail(d, mx, my, bx, by - 1, blk_idx), left = lavail(d, mx, my, bx - 1, by, blk_idx);
    int ul = lavail(d, mx, my, bx - 1, by - 1, blk_idx);
    int ur = lavail(d, mx, my, bx + 4, by - 1, blk_idx);
    if (blk_idx == 3 || blk_idx == 11 || blk_idx == 7 || blk_idx == 13 || blk_idx == 15) ur = 0;
    if ((blk_idx == 5) && !avail_mb(d, mx + 1, my - 1, mx, my)) ur = 0;
    int p[13];                           /* p[0] = (-1,-1), p[1..8] = (0..7,-1), p[9..12] = (-1,0..3) */
    p[0] = ul ? R[(Y - 1) * W + X - 1] : 0;
    for (int i = 0; i < 4; i++) p[1 + i] = up ? R[(Y - 1) * W + X + i] : 0;
    for (int i = 4; i < 8; i++) p[1 + i] = up ? (ur ? R[(Y - 1) * W + X + i] : p[4]) : 0;
    for (int i = 0; i < 4; i++) p[9 + i] = left ? R[(Y + i) * W + X - 1] : 0;
#define T(x) p[1 + (x)]
#define L(y) ((y) < 0 ? p[0] : p[9 + (y)])
    *ok = 1;
    if ((mode == 0 || mode == 3 || mode == 7) && !up) *ok = 0;
    if ((mode == 1 || mode == 8) && !left) *ok = 0;
    if ((mode == 4 || mode == 5 || mode == 6) && !(up && left && ul)) *ok = 0;
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) {
            int v = 0;
            switch (mode) {
            case 0: v = T(x); break;
            case 1: v = L(y); break;
            case 2:
                if (up && left) v = (T(0) + T(1) + T(2) + T(3) + L(0) + L(1) + L(2) + L(3) + 4) >> 3;
                else if (left) v = (L(0) + L(1) + L(2) + L(3) + 2) >> 2;
                else if (up) v = (T(0) + T(1) + T(2) + T(3) + 2) >> 2;
                else v = 128;
                break;
            case 3: v = (x == 3 && y == 3) ? (T(6) + 3 * T(7) + 2) >> 2 : (T(x + y) + 2 * T(x + y + 1) + T(x + y + 2) + 2) >> 2; break;
            case 4:
                if (x > y) v = (T(x - y - 2) + 2 * T(x - y - 1) + T(x - y) + 2) >> 2;
                else if (x < y) v = (L(y - x - 2) + 2 * L(y - x - 1) + L(y - x) + 2) >> 2;
                else v = (T(0) + 2 * p[0] + L(0) + 2) >> 2;
                break;
            case 5: {
                int z = 2 * x - y;
                if (z >= 0 && !(z & 1)) v = (T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 1) >> 1;
                else if (z >= 0) v = (T(x - (y >> 1) - 2) + 2 * T(x - (y >> 1) - 1) + T(x - (y >> 1)) + 2) >> 2;
                else if (z == -1) v = (L(0) + 2 * p[0] + T(0) + 2) >> 2;
                else v = (L(y - 1) + 2 * L(y - 2) + L(y - 3) + 2) >> 2;
                break;
            }
            case 6: {
                int z = 2 * y - x;
                if (z >= 0 && !(z & 1)) v = (L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 1) >> 1;
                else if (z >= 0) v = (L(y - (x >> 1) - 2) + 2 * L(y - (x >> 1) - 1) + L(y - (x >> 1)) + 2) >> 2;
                else if (z == -1) v = (L(0) + 2 * p[0] + T(0) + 2) >> 2;
                else v = (T(x - 1) + 2 * T(x - 2) + T(x - 3) + 2) >> 2;
                break;
            }
            case 7:
                v = (y & 1) ? (T(x + (y >> 1)) + 2 * T(x + (y >> 1) + 1) + T(x + (y >> 1) + 2) + 2) >> 2
                            : (T(x + (y >> 1)) + T(x + (y >> 1) + 1) + 1) >> 1;
                break;
            case 8: {
                int z = x + 2 * y;
                if (z > 5) v = L(3);
                else if (z == 5) v = (L(2) + 3 * L(3) + 2) >> 2;
                else if (!(z & 1)) v = (L(y + (x >> 1)) + L(y + (x >> 1) + 1) + 1) >> 1;
                else v = (L(y + (x >> 1)) + 2 * L(y + (x >> 1) + 1) + L(y + (x >> 1) + 2) + 2) >> 2;
                break;
            }
            }
            pr[4 * y + x] = (uint8_t)v;
        }
#undef T
#undef L
}
static int pred16(const jmo_dec *d, int mx, int my, int mode, uint8_t *pr) {
    const uint8_t *R = d->cur[0];
    int W = d->W, X = 16 * mx, Y = 16 * my;
    int up = avail_mb(d, mx, my - 1, mx, my), left = avail_mb(d, mx - 1, my, mx, my), ul = avail_mb(d, mx - 1, my - 1, mx, my);
    int T[17], L[17];                   /* index 0 = corner */
    T[0] = L[0] = ul ? R[(Y - 1) * W + X - 1] : 0;
    for (int i = 0; i < 16; i++) { T[1 + i] = up ? R[(Y - 1) * W + X + i] : 0; L[1 + i] = left ? R[(Y + i) * W + X - 1] : 0; }
    if (mode == 0 && !up) return -1;
    if (mode == 1 && !left) return -1;
    if (mode == 3 && !(up && left && ul)) return -1;
    int st = 0, sl = 0;
    for (int i = 1; i <= 16; i++) { st += T[i]; sl += L[i]; }
    int dc = (up && left) ? (st + sl + 16) >> 5 : up ? (st + 8) >> 4 : left ? (sl + 8) >> 4 : 128;
    int H = 0, V = 0;
    for (int xp = 0; xp < 8; xp++) { H += (xp + 1) * (T[1 + 8 + xp] - T[1 + 6 - xp]); V += (xp + 1) * (L[1 + 8 + xp] - L[1 + 6 - xp]); }
    int a = 16 * (L[16] + T[16]), bb = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) {
            int v = mode == 0 ? T[1 + x] : mode == 1 ? L[1 + y] : mode == 2 ? dc : clip255((a + bb * (x - 7) + c * (y - 7) + 16) >> 5);
            pr[16 * y + x] = (uint8_t)v;
        }
    return 0;
}
static int predc(const jmo_dec *d, int mx, int my, int comp, int mode, uint8_t *pr) {
    const uint8_t *R = d->cur[comp];
    int W = d->W / 2, X = 8 * mx, Y = 8 * my;
    int up = avail_mb(d, mx, my - 1, mx, my), left = avail_mb(d, mx - 1, my, mx, my), ul = avail_mb(d, mx - 1, my - 1, mx, my);
    int T[9], L[9];
    T[0] = L[0] = ul ? R[(Y - 1) * W + X - 1] : 0;
    for (int i = 0; i < 8; i++) { T[1 + i] = up ? R[(Y - 1) * W + X + i] : 0; L[1 + i] = left ? R[(Y + i) * W + X - 1] : 0; }
    if (mode == 1 && !left) return -1;
    if (mode == 2 && !up) return -1;
    if (mode == 3 && !(up && left && ul)) return -1;
    for (int b = 0; b < 4; b++) {
        int xo = (b & 1) * 4, yo = (b >> 1) * 4, v = 0;
        if (mode == 0) {
            int su = 0, sv = 0;
            for (int i = 0; i < 4; i++) { su += T[1 + xo + i]; sv += L[1 + yo + i]; }
            if ((xo == 0 && yo == 0) || (xo > 0 && yo > 0)) v = (up && left) ? (su + sv + 4) >> 3 : left ? (sv + 2) >> 2 : up ? (su + 2) >> 2 : 128;
            else if (xo > 0) v = up ? (su + 2) >> 2 : left ? (sv + 2) >> 2 : 128;
            else v = left ? (sv + 2) >> 2 : up ? (su + 2) >> 2 : 128;
        }
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                int xx = xo + x, yy = yo + y, w = v;
                if (mode == 1) w = L[1 + yy];
                else if (mode == 2) w = T[1 + xx];
                else if (mode == 3) {
                    int H = 0, V = 0;
                    for (int xp = 0; xp < 4; xp++) { H += (xp + 1) * (T[1 + 4 + xp] - T[1 + 2 - xp]); V += (xp + 1) * (L[1 + 4 + xp] - L[1 + 2 - xp]); }
                    int a = 16 * (L[8] + T[8]), bb = (34 * H + 32) >> 6, c = (34 * V + 32) >> 6;
                    w = clip255((a + bb * (xx - 3) + c * (yy - 3) + 16) >> 5);
                }
                pr[8 * yy + xx] = (uint8_t)w;
            }
    }
    return 0;
}

/* ---- scaling + inverse transform (8.5) ------------------------------------------------- */
static const int normA[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
static int lscale(int qm, int pos) {       /* LevelScale4x4 = 16 * normAdjust (flat) */
    int x = pos & 3, y = pos >> 2;
    int cls = (!(x & 1) && !(y & 1)) ? 0 : ((x & 1) && (y & 1)) ? 1 : 2;
    return 16 * normA[qm][cls];
}
static void scale4x4(int32_t *c, int qp, int skip_dc) {
    for (int k = skip_dc; k < 16; k++) {
        int ls = lscale(qp % 6, k);
        if (qp >= 24) c[k] = c[k] * ls * (1 << (qp / 6 - 4));
        else c[k] = (c[k] * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
    }
}
static void recon4x4(int32_t *c, const uint8_t *pred, int ps, uint8_t *out, int os) {
    int32_t r[16];
    jmo_inverse4x4(c, r);
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) out[y * os + x] = (uint8_t)clip255(pred[y * ps + x] + ((r[4 * y + x] + 32) >> 6));
}

/* ---- Intra_8x8 (8.3.2.2): the 25 reference samples as one edge e[0..24] running from
 * p[-1,7] up to p[-1,0] (e[7-y]), the corner p[-1,-1] (e[8]) and along p[0..15,-1] (e[9+x]);
 * the 8.3.2.2.1 filter is a [1 2 1] tap along the edge whose missing outer neighbour is
 * replaced by the centre sample, and every directional mode reads that filtered edge. */
static int pred8x8(const jmo_dec *d, int mx, int my, int b8, int mode, uint8_t *pr) {
    const uint8_t *R = d->cur[0];
    int W = d->W, bx = 8 * (b8 & 1), by = 8 * (b8 >> 1), X = 16 * mx + bx, Y = 16 * my + by;
    int left = bx ? 1 : avail_mb(d, mx - 1, my, mx, my);
    int up = by ? 1 : avail_mb(d, mx, my - 1, mx, my);
    int ul = bx && by ? 1 : bx ? avail_mb(d, mx, my - 1, mx, my) : by ? avail_mb(d, mx - 1, my, mx, my) : avail_mb(d, mx - 1, my - 1, mx, my);
    int ur = b8 == 0 ? avail_mb(d, mx, my - 1, mx, my) : b8 == 1 ? avail_mb(d, mx + 1, my - 1, mx, my) : b8 == 2;
    int e[25], av[25], f[25];
    for (int i = 0; i < 25; i++) { e[i] = 0; av[i] = 0; }
    for (int y = 0; y < 8; y++) if (left) { e[7 - y] = R[(Y + y) * W + X - 1]; av[7 - y] = 1; }
    if (ul) { e[8] = R[(Y - 1) * W + X - 1]; av[8] = 1; }
    for (int x = 0; x < 16; x++)
        if (up) { e[9 + x] = x < 8 || ur ? R[(Y - 1) * W + X + x] : R[(Y - 1) * W + X + 7]; av[9 + x] = 1; }
    for (int i = 0; i < 25; i++) {
        if (!av[i]) continue;
        int l = i > 0 && av[i - 1] ? e[i - 1] : e[i], r = i < 24 && av[i + 1] ? e[i + 1] : e[i];
        f[i] = (l + 2 * e[i] + r + 2) >> 2;
    }
#define TT(x) f[9 + (x)]
#define LL(y) f[7 - (y)]
#define TAP(c) ((f[(c) - 1] + 2 * f[c] + f[(c) + 1] + 2) >> 2)
    if (((mode == 0 || mode == 3 || mode == 7) && !up) || ((mode == 1 || mode == 8) && !left) ||
        ((mode == 4 || mode == 5 || mode == 6) && !(up && left && ul)))
        return -1;
    int dc = 128, st = 0, sl = 0;
    for (int i = 0; i < 8; i++) { st += up ? TT(i) : 0; sl += left ? LL(i) : 0; }
    if (up && left) dc = (st + sl + 8) >> 4;
    else if (up) dc = (st + 4) >> 3;
    else if (left) dc = (sl + 4) >> 3;
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            int v = dc, z;
            switch (mode) {
            case 0: v = TT(x); break;
            case 1: v = LL(y); break;
            case 3: v = x + y < 14 ? TAP(10 + x + y) : (f[23] + 3 * f[24] + 2) >> 2; break;
            case 4: v = TAP(8 + x - y); break;
            case 5:
                z = 2 * x - y;
                if (z >= 0 && !(z & 1)) v = (f[8 + x - (y >> 1)] + f[9 + x - (y >> 1)] + 1) >> 1;
                else if (z > 0) v = TAP(8 + x - (y >> 1));
                else v = TAP(9 + z);
                break;
            case 6:
                z = 2 * y - x;
                if (z >= 0 && !(z & 1)) v = (f[8 - y + (x >> 1)] + f[7 - y + (x >> 1)] + 1) >> 1;
                else if (z > 0) v = TAP(8 - y + (x >> 1));
                else v = TAP(7 - z);
                break;
            case 7:
                v = (y & 1) ? (TT(x + (y >> 1)) + 2 * TT(x + (y >> 1) + 1) + TT(x + (y >> 1) + 2) + 2) >> 2
                            : (TT(x + (y >> 1)) + TT(x + (y >> 1) + 1) + 1) >> 1;
                break;
            case 8:
                z = x + 2 * y;
                if (z > 13) v = LL(7);
                else if (z == 13) v = (LL(6) + 3 * LL(7) + 2) >> 2;
                else if (!(z & 1)) v = (LL(y + (x >> 1)) + LL(y + (x >> 1) + 1) + 1) >> 1;
                else v = (LL(y + (x >> 1)) + 2 * LL(y + (x >> 1) + 1) + LL(y + (x >> 1) + 2) + 2) >> 2;
                break;
            }
            pr[8 * y + x] = (uint8_t)v;
        }
#undef TT
#undef LL
#undef TAP
    return 0;
}
/* 8x8 frame zig-zag (Table 8-13, 8x8 field omitted) as (x, y) pairs */
static const uint8_t zz8[64][2] = {
    {0, 0}, {1, 0}, {0, 1}, {0, 2}, {1, 1}, {2, 0}, {3, 0}, {2, 1}, {1, 2}, {0, 3}, {0, 4}, {1, 3}, {2, 2},
    {3, 1}, {4, 0}, {5, 0}, {4, 1}, {3, 2}, {2, 3}, {1, 4}, {0, 5}, {0, 6}, {1, 5}, {2, 4}, {3, 3}, {4, 2},
    {5, 1}, {6, 0}, {7, 0}, {6, 1}, {5, 2}, {4, 3}, {3, 4}, {2, 5}, {1, 6}, {0, 7}, {1, 7}, {2, 6}, {3, 5},
    {4, 4}, {5, 3}, {6, 2}, {7, 1}, {7, 2}, {6, 3}, {5, 4}, {4, 5}, {3, 6}, {2, 7}, {3, 7}, {4, 6}, {5, 5},
    {6, 4}, {7, 3}, {7, 4}, {6, 5}, {5, 6}, {4, 7}, {5, 7}, {6, 6}, {7, 5}, {7, 6}, {6, 7}, {7, 7}};
/* LevelScale8x8 = 16 * normAdjust8x8 (8.5.9, flat Default weights) and 8.5.13.1 scaling */
static int lscale8(int qm, int i, int j) {
    static const int v8[6][6] = {{20, 18, 32, 19, 25, 24}, {22, 19, 35, 21, 28, 26}, {26, 23, 42, 24, 33, 31},
                                 {28, 25, 45, 26, 35, 33}, {32, 28, 51, 30, 40, 38}, {36, 32, 58, 34, 46, 43}};
    int k = (i % 4 == 0 && j % 4 == 0) ? 0 : (i % 2 == 1 && j % 2 == 1) ? 1 : (i % 4 == 2 && j % 4 == 2) ? 2
          : ((i % 4 == 0 && j % 2 == 1) || (i % 2 == 1 && j % 4 == 0)) ? 3
          : ((i % 4 == 0 && j % 4 == 2) || (i % 4 == 2 && j % 4 == 0)) ? 4 : 5;
    return 16 * v8[qm][k];
}
static void recon8x8(const int *c64, int qp, const uint8_t *pred, int ps, uint8_t *out, int os) {
    int32_t m[64], r[64];
    for (int k = 0; k < 64; k++) {
        int x = zz8[k][0], y = zz8[k][1], ls = lscale8(qp % 6, y, x), c = c64[k];
        m[8 * y + x] = qp >= 36 ? c * ls * (1 << (qp / 6 - 6)) : (c * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
    jmo_inverse8x8(m, r);
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) out[y * os + x] = (uint8_t)clip255(pred[y * ps + x] + ((r[8 * y + x] + 32) >> 6));
}

/* ---- inter prediction (8.4.2.2) ------------------------------------------------------- */
static void inter_pred(const jmo_dec *d, int mx, int my, const int16_t mv16[16][2], uint8_t *py, uint8_t *pu, uint8_t *pv) {
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) {
            const int16_t *v = mv16[(y >> 2) * 4 + (x >> 2)];
            py[16 * y + x] = (uint8_t)jmo_luma_qpel_sample(d->ref[0], d->W, d->H, d->W, 4 * (16 * mx + x) + v[0], 4 * (16 * my + y) + v[1]);
        }
    int Wc = d->W / 2, Hc = d->H / 2;
    for (int c = 1; c <= 2; c++)
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                const int16_t *v = mv16[(y >> 1) * 4 + (x >> 1)];
                int xi = 8 * mx + x + (v[0] >> 3), yi = 8 * my + y + (v[1] >> 3), fx = v[0] & 7, fy = v[1] & 7;
                const uint8_t *R = d->ref[c];
                int A = R[iclip(0, Hc - 1, yi) * Wc + iclip(0, Wc - 1, xi)], B = R[iclip(0, Hc - 1, yi) * Wc + iclip(0, Wc - 1, xi + 1)];
                int C = R[iclip(0, Hc - 1, yi + 1) * Wc + iclip(0, Wc - 1, xi)], D = R[iclip(0, Hc - 1, yi + 1) * Wc + iclip(0, Wc - 1, xi + 1)];
                (c == 1 ? pu : pv)[8 * y + x] = (uint8_t)(((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6);
            }
}

/* ---- motion vector prediction (8.4.1.3) using "already decoded" partition tracking ------ */
static int nb4(const jmo_dec *d, int mx, int my, int xN, int yN, int *idx) {
    int tx, ty;
    if (yN > 15) return 0;
    if (xN < 0) { tx = mx - 1; ty = yN < 0 ? my - 1 : my; }
    else if (xN <= 15) { tx = mx; ty = yN < 0 ? my - 1 : my; }
    else { if (yN >= 0) return 0; tx = mx + 1; ty = my - 1; }
    if (tx < 0 || ty < 0 || tx >= d->mbw || ty * d->mbw + tx < d->slice_first) return 0;
    int W4 = d->W / 4;
    int i = ((16 * my + yN) >> 2) * W4 + ((16 * mx + xN) >> 2);
    if (tx == mx && ty == my && !d->dec4[i]) return 0;   /* not yet decoded partition */
    *idx = i;
    return 1;
}
static void mvpred(const jmo_dec *d, int mx, int my, int x, int y, int w, int h, int refidx, int *pmv) {
    int ia = 0, ib = 0, ic = 0;
    int aa = nb4(d, mx, my, x - 1, y, &ia), ab = nb4(d, mx, my, x, y - 1, &ib), ac = nb4(d, mx, my, x + w, y - 1, &ic);
    if (!ac) ac = nb4(d, mx, my, x - 1, y - 1, &ic);
    int rA = aa ? d->refi[ia] : -1, rB = ab ? d->refi[ib] : -1, rC = ac ? d->refi[ic] : -1;
    int mA[2] = {aa ? d->mv[2 * ia] : 0, aa ? d->mv[2 * ia + 1] : 0};
    int mB[2] = {ab ? d->mv[2 * ib] : 0, ab ? d->mv[2 * ib + 1] : 0};
    int mC[2] = {ac ? d->mv[2 * ic] : 0, ac ? d->mv[2 * ic + 1] : 0};
    if (w == 16 && h == 8) {
        if (y == 0 && rB == refidx) { pmv[0] = mB[0]; pmv[1] = mB[1]; return; }
        if (y == 8 && rA == refidx) { pmv[0] = mA[0]; pmv[1] = mA[1]; return; }
    } else if (w == 8 && h == 16) {
        if (x == 0 && rA == refidx) { pmv[0] = mA[0]; pmv[1] = mA[1]; return; }
        if (x == 8 && rC == refidx) { pmv[0] = mC[0]; pmv[1] = mC[1]; return; }
    }
    if (!ab && !ac && aa) { rB = rC = rA; mB[0] = mC[0] = mA[0]; mB[1] = mC[1] = mA[1]; }
    int n = (rA == refidx) + (rB == refidx) + (rC == refidx);
    for (int k = 0; k < 2; k++) {
        if (n == 1) pmv[k] = rA == refidx ? mA[k] : rB == refidx ? mB[k] : mC[k];
        else pmv[k] = mA[k] + mB[k] + mC[k] - imin(mA[k], imin(mB[k], mC[k])) - imax(mA[k], imax(mB[k], mC[k]));
    }
}
static void set_part(jmo_dec *d, int mx, int my, int x, int y, int w, int h, int mvx, int mvy, int refidx, int16_t mv16[16][2]) {
    int W4 = d->W / 4;
    for (int yy = y; yy < y + h; yy += 4)
        for (int xx = x; xx < x + w; xx += 4) {
            int i = ((16 * my + yy) >> 2) * W4 + ((16 * mx + xx) >> 2);
            d->mv[2 * i] = (int16_t)mvx; d->mv[2 * i + 1] = (int16_t)mvy; d->refi[i] = (int8_t)refidx; d->dec4[i] = 1;
            mv16[(yy >> 2) * 4 + (xx >> 2)][0] = (int16_t)mvx; mv16[(yy >> 2) * 4 + (xx >> 2)][1] = (int16_t)mvy;
        }
}

/* ---- nC (9.2.1) ------------------------------------------------------------------------ */
static int calc_nc(const jmo_dec *d, int mx, int my, int comp, int x4, int y4, const uint8_t *cur) {
    int st = comp ? 2 : 4, base = comp ? 16 + 4 * (comp - 1) : 0, lim = st - 1;
    int na = 0, nb = 0, aa = 0, ab = 0;
    if (x4 > 0) { aa = 1; na = cur[base + y4 * st + x4 - 1]; }
    else if (avail_mb(d, mx - 1, my, mx, my)) { aa = 1; na = d->mi[my * d->mbw + mx - 1].tc[base + y4 * st + lim]; }
    if (y4 > 0) { ab = 1; nb = cur[base + (y4 - 1) * st + x4]; }
    else if (avail_mb(d, mx, my - 1, mx, my)) { ab = 1; nb = d->mi[(my - 1) * d->mbw + mx].tc[base + lim * st + x4]; }
    return (aa && ab) ? (na + nb + 1) >> 1 : aa ? na : ab ? nb : 0;
}

static const int zz[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
static const int QPCt[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
                             26, 27, 28, 29, 29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

#define FAIL(...) do { snprintf(d->err, sizeof d->err, __VA_ARGS__); return -1; } while (0)

static int decode_mb(jmo_dec *d, br_t *b, int mx, int my, int slice_p, int mbt_ue, int skip, int *qp) {
    mbinfo *mi = &d->mi[my * d->mbw + mx];
    memset(mi, 0, sizeof(*mi));
    int W4 = d->W / 4;
    for (int k = 0; k < 16; k++) { int i = (4 * my + (k >> 2)) * W4 + 4 * mx + (k & 3); d->dec4[i] = 0; d->refi[i] = -1; d->mv[2 * i] = d->mv[2 * i + 1] = 0; }
    int16_t mv16[16][2];
    memset(mv16, 0, sizeof(mv16));
    uint8_t pred[256], predu[64], predv[64];
    int i16mode = 0, cbp = 0, intra_type = -1;    /* intra_type: -1 inter, 0 I_NxN, 1 I16 */
    int no_sub8x8 = 0;
    int ipm[16];
    if (skip) {
        mi->mbtype = 3;
        int ia = 0, ib = 0;
        int aa = nb4(d, mx, my, -1, 0, &ia), ab = nb4(d, mx, my, 0, -1, &ib);
        int mvx = 0, mvy = 0;
        if (aa && ab && !(d->refi[ia] == 0 && !d->mv[2 * ia] && !d->mv[2 * ia + 1]) && !(d->refi[ib] == 0 && !d->mv[2 * ib] && !d->mv[2 * ib + 1])) {
            int p[2];
            mvpred(d, mx, my, 0, 0, 16, 16, 0, p);
            mvx = p[0]; mvy = p[1];
        }
        set_part(d, mx, my, 0, 0, 16, 16, mvx, mvy, 0, mv16);
    } else {
        int t = mbt_ue;
        if (slice_p) { if (t >= 5) { t -= 5; intra_type = t == 0 ? 0 : 1; } }
        else intra_type = t == 0 ? 0 : 1;
        if (intra_type == 1) {
            if (t > 24) FAIL("I_PCM unsupported");
            i16mode = (t - 1) % 4;
            cbp = (((t - 1) / 4) % 3) << 4 | ((t >= 13) ? 15 : 0);
        }
        if (intra_type >= 0) {
            mi->intra = 1;
            mi->mbtype = intra_type == 0 ? 1 : 2;
            if (intra_type == 0 && d->t8mode) mi->t8 = rb(b);
            if (mi->t8) {                               /* Intra_8x8: predIntra8x8PredMode (8.3.2.1) */
                mi->mbtype = 4;
                int m8[4];
                for (int b8 = 0; b8 < 4; b8++) {
                    int x4 = (b8 & 1) * 2, y4 = (b8 >> 1) * 2;
                    int flag = rb(b), rem = flag ? 0 : (int)rbits(b, 3);
                    int ma = -1, mb = -1, dcp = 0;
                    if (x4 > 0) ma = m8[b8 - 1];
                    else if (avail_mb(d, mx - 1, my, mx, my)) { const mbinfo *n = &d->mi[my * d->mbw + mx - 1]; ma = (n->mbtype == 1 || n->mbtype == 4) ? n->ipm[y4 * 4 + 3] : 2; }
                    else dcp = 1;
                    if (y4 > 0) mb = m8[b8 - 2];
                    else if (avail_mb(d, mx, my - 1, mx, my)) { const mbinfo *n = &d->mi[(my - 1) * d->mbw + mx]; mb = (n->mbtype == 1 || n->mbtype == 4) ? n->ipm[12 + x4] : 2; }
                    else dcp = 1;
                    int pm = dcp ? 2 : imin(ma, mb);
                    m8[b8] = flag ? pm : (rem < pm ? rem : rem + 1);
                }
                for (int k = 0; k < 16; k++) { ipm[k] = m8[((k >> 3) << 1) + ((k & 3) >> 1)]; mi->ipm[k] = (int8_t)ipm[k]; }
            } else if (intra_type == 0) {
                for (int blk = 0; blk < 16; blk++) {
                    int x4 = ((blk >> 2) & 1) * 2 + (blk & 1), y4 = (blk >> 3) * 2 + ((blk >> 1) & 1);
                    int flag = rb(b), rem = flag ? 0 : (int)rbits(b, 3);
                    /* predIntra4x4PredMode (8.3.1.1) */
                    int ma = -1, mb = -1, dcp = 0;
                    if (x4 > 0) ma = ipm[y4 * 4 + x4 - 1];
                    else if (avail_mb(d, mx - 1, my, mx, my)) { const mbinfo *n = &d->mi[my * d->mbw + mx - 1]; ma = (n->mbtype == 1 || n->mbtype == 4) ? n->ipm[y4 * 4 + 3] : 2; }
                    else dcp = 1;
                    if (y4 > 0) mb = ipm[(y4 - 1) * 4 + x4];
                    else if (avail_mb(d, mx, my - 1, mx, my)) { const mbinfo *n = &d->mi[(my - 1) * d->mbw + mx]; mb = (n->mbtype == 1 || n->mbtype == 4) ? n->ipm[12 + x4] : 2; }
                    else dcp = 1;
                    int pm = dcp ? 2 : imin(ma, mb);
                    ipm[y4 * 4 + x4] = flag ? pm : (rem < pm ? rem : rem + 1);
                }
                memcpy(mi->ipm, (int8_t[16]){0}, 16);
                for (int k = 0; k < 16; k++) mi->ipm[k] = (int8_t)ipm[k];
            }
            int cmode = rue(b);
            if (cmode > 3) FAIL("bad chroma mode");
            if (predc(d, mx, my, 1, cmode, predu) || predc(d, mx, my, 2, cmode, predv)) FAIL("chroma pred mode %d unavailable at MB %d,%d", cmode, mx, my);
            if (intra_type == 1 && pred16(d, mx, my, i16mode, pred)) FAIL("I16 mode %d unavailable at MB %d,%d", i16mode, mx, my);
        } else {
            mi->mbtype = 0;
            if (t > 4) FAIL("bad P mb_type %d", t);
            no_sub8x8 = 1;
            if (t == 3 || t == 4) {
                int sub[4];
                for (int i = 0; i < 4; i++) { sub[i] = rue(b); if (sub[i] > 3) FAIL("bad sub_mb_type"); if (sub[i]) no_sub8x8 = 0; }
                if (d->num_ref_l0 > 1) FAIL("multiple refs unsupported");
                for (int i = 0; i < 4; i++) {
                    int ox = (i & 1) * 8, oy = (i >> 1) * 8;
                    int sw = sub[i] == 0 || sub[i] == 1 ? 8 : 4, sh = sub[i] == 0 || sub[i] == 2 ? 8 : 4;
                    for (int y = 0; y < 8; y += sh)
                        for (int x = 0; x < 8; x += sw) {
                            int p[2];
                            mvpred(d, mx, my, ox + x, oy + y, sw, sh, 0, p);
                            int dx = rse(b), dy = rse(b);
                            set_part(d, mx, my, ox + x, oy + y, sw, sh, p[0] + dx, p[1] + dy, 0, mv16);
                        }
                }
            } else {
                if (d->num_ref_l0 > 1) FAIL("multiple refs unsupported");
                int np = t == 0 ? 1 : 2, w = t == 2 ? 8 : 16, h = t == 1 ? 8 : 16;
                for (int pi = 0; pi < np; pi++) {
                    int x = t == 2 ? 8 * pi : 0, y = t == 1 ? 8 * pi : 0, p[2];
                    mvpred(d, mx, my, x, y, w, h, 0, p);
                    int dx = rse(b), dy = rse(b);
                    set_part(d, mx, my, x, y, w, h, p[0] + dx, p[1] + dy, 0, mv16);
                }
            }
        }
        if (intra_type != 1) {
            int code = rue(b);
            if (code > 47) FAIL("bad cbp code");
            cbp = intra_type == 0 ? cbp_intra[code] : cbp_inter[code];
            if (intra_type < 0 && (cbp & 15) && d->t8mode && no_sub8x8) mi->t8 = rb(b);
        }
        if (cbp > 0 || intra_type == 1) {
            int dq = rse(b);
            *qp = (*qp + dq + 52) % 52;
        }
    }
    mi->qp = *qp;
    if (!mi->intra) inter_pred(d, mx, my, mv16, pred, predu, predv);
    /* ---- residual + reconstruction ---- */
    int qp_ = *qp, qpc = QPCt[iclip(0, 51, qp_ + d->cqp_off)];
    int cbpl = cbp & 15, cbpc = cbp >> 4;
    int32_t dcY[16] = {0};
    uint8_t *RY = d->cur[0];
    int W = d->W;
    if (intra_type == 1) {
        int c[16];
        if (read_block(b, calc_nc(d, mx, my, 0, 0, 0, mi->tc), 16, c) < 0) FAIL("I16 DC at %d,%d", mx, my);
        int32_t m[16], t2[16];
        for (int k = 0; k < 16; k++) m[zz[k]] = c[k];
        for (int y = 0; y < 4; y++) {
            int32_t *r = m + 4 * y;
            int e0 = r[0] + r[1] + r[2] + r[3], e1 = r[0] + r[1] - r[2] - r[3], e2 = r[0] - r[1] - r[2] + r[3], e3 = r[0] - r[1] + r[2] - r[3];
            t2[4 * y] = e0; t2[4 * y + 1] = e1; t2[4 * y + 2] = e2; t2[4 * y + 3] = e3;
        }
        for (int x = 0; x < 4; x++) {
            int a0 = t2[x], a1 = t2[4 + x], a2 = t2[8 + x], a3 = t2[12 + x];
            int f[4] = {a0 + a1 + a2 + a3, a0 + a1 - a2 - a3, a0 - a1 - a2 + a3, a0 - a1 + a2 - a3};
            for (int y = 0; y < 4; y++) {
                int ls = lscale(qp_ % 6, 0);
                int v = qp_ >= 36 ? f[y] * ls * (1 << (qp_ / 6 - 6)) : (f[y] * ls + (1 << (5 - qp_ / 6))) >> (6 - qp_ / 6);
                dcY[4 * y + x] = v;
            }
        }
    }
    for (int b8 = 0; b8 < 4 && mi->t8; b8++) {       /* 8x8 transform: 4 interleaved CAVLC blocks */
        int c64[64] = {0}, any = 0;
        for (int i4 = 0; i4 < 4; i4++) {
            int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1), c[16] = {0}, tc = 0;
            if (cbpl & (1 << b8)) {
                tc = read_block(b, calc_nc(d, mx, my, 0, x4, y4, mi->tc), 16, c);
                if (tc < 0) FAIL("luma 8x8 block %d at MB %d,%d", b8, mx, my);
            }
            mi->tc[y4 * 4 + x4] = (uint8_t)tc;
            for (int k = 0; k < 16; k++) { c64[4 * k + i4] = c[k]; any |= c[k] != 0; }
        }
        int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
        if (any) mi->nzblk |= 0x33 << ((by >> 2) * 4 + (bx >> 2));
        uint8_t *dst = RY + (16 * my + by) * W + 16 * mx + bx;
        if (intra_type == 0) {
            uint8_t p64[64];
            if (pred8x8(d, mx, my, b8, ipm[(by >> 2) * 4 + (bx >> 2)], p64)) FAIL("I8 mode unavailable at MB %d,%d", mx, my);
            recon8x8(c64, qp_, p64, 8, dst, W);
        } else recon8x8(c64, qp_, pred + by * 16 + bx, 16, dst, W);
    }
    for (int blk = 0; blk < 16 && !mi->t8; blk++) {
        int b8 = blk >> 2;
        int x4 = (b8 & 1) * 2 + (blk & 1), y4 = (b8 >> 1) * 2 + ((blk >> 1) & 1);
        int c[16] = {0};
        int tc = 0;
        if (cbpl & (1 << b8)) {
            int nC = calc_nc(d, mx, my, 0, x4, y4, mi->tc);
            if (intra_type == 1) { int c15[15]; tc = read_block(b, nC, 15, c15); for (int k = 0; k < 15; k++) c[k + 1] = c15[k]; }
            else tc = read_block(b, nC, 16, c);
            if (tc < 0) FAIL("luma block %d at MB %d,%d", blk, mx, my);
        }
        mi->tc[y4 * 4 + x4] = (uint8_t)tc;
        int any = 0;
        for (int k = 0; k < 16; k++) any |= c[k] != 0;
        if (any) mi->nzblk |= 1 << (y4 * 4 + x4);
        int32_t m[16];
        for (int k = 0; k < 16; k++) m[zz[k]] = c[k];
        scale4x4(m, qp_, intra_type == 1);
        if (intra_type == 1) m[0] = dcY[y4 * 4 + x4];
        uint8_t *dst = RY + (16 * my + 4 * y4) * W + 16 * mx + 4 * x4;
        if (intra_type == 0) {
            uint8_t p4[16];
            int ok;
            pred4x4(d, mx, my, 4 * x4, 4 * y4, blk, ipm[y4 * 4 + x4], p4, &ok);
            if (!ok) FAIL("I4 mode %d unavailable at MB %d,%d blk %d", ipm[y4 * 4 + x4], mx, my, blk);
            recon4x4(m, p4, 4, dst, W);
        } else recon4x4(m, pred + 4 * y4 * 16 + 4 * x4, 16, dst, W);
    }
    /* chroma */
    int dcc[2][4] = {{0}};
    if (cbpc) {
        for (int comp = 0; comp < 2; comp++) {
            int c[4];
            if (read_block(b, -1, 4, c) < 0) FAIL("chroma DC");
            int f[4] = {c[0] + c[1] + c[2] + c[3], c[0] - c[1] + c[2] - c[3], c[0] + c[1] - c[2] - c[3], c[0] - c[1] - c[2] + c[3]};
            for (int k = 0; k < 4; k++) dcc[comp][k] = (f[k] * lscale(qpc % 6, 0) * (1 << (qpc / 6))) >> 5;
        }
    }
    for (int comp = 0; comp < 2; comp++) {
        uint8_t *R = d->cur[1 + comp];
        int Wc = d->W / 2;
        for (int k = 0; k < 4; k++) {
            int c[16] = {0}, tc = 0;
            if (cbpc == 2) {
                int c15[15];
                tc = read_block(b, calc_nc(d, mx, my, 1 + comp, k & 1, k >> 1, mi->tc), 15, c15);
                if (tc < 0) FAIL("chroma AC");
                for (int q = 0; q < 15; q++) c[q + 1] = c15[q];
            }
            mi->tc[16 + 4 * comp + k] = (uint8_t)tc;
            int32_t m[16];
            for (int q = 0; q < 16; q++) m[zz[q]] = c[q];
            scale4x4(m, qpc, 1);
            m[0] = dcc[comp][k];
            int xo = (k & 1) * 4, yo = (k >> 1) * 4;
            recon4x4(m, (comp ? predv : predu) + yo * 8 + xo, 8, R + (8 * my + yo) * Wc + 8 * mx + xo, Wc);
        }
    }
    return b->err ? -1 : 0;
}

/* ---- deblocking (8.7), independent restatement ------------------------------------------ */
static const int Alpha[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 5, 6, 7, 8, 9, 10, 12, 13,
                              15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
static const int Beta[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4,
                             6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
static const int Tc0[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1},
    {1, 1, 1}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4}, {2, 3, 4}, {3, 3, 5}, {3, 4, 6},
    {3, 4, 6}, {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11}, {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

static int bs_of(const jmo_dec *d, int xp, int yp, int xq, int yq, int mbedge) {  /* luma sample coords */
    const mbinfo *P = &d->mi[(yp >> 4) * d->mbw + (xp >> 4)], *Q = &d->mi[(yq >> 4) * d->mbw + (xq >> 4)];
    if (P->intra || Q->intra) return mbedge ? 4 : 3;
    int bp = ((yp & 15) >> 2) * 4 + ((xp & 15) >> 2), bq = ((yq & 15) >> 2) * 4 + ((xq & 15) >> 2);
    if (((P->nzblk >> bp) & 1) || ((Q->nzblk >> bq) & 1)) return 2;
    int W4 = d->W / 4, ip = (yp >> 2) * W4 + (xp >> 2), iq = (yq >> 2) * W4 + (xq >> 2);
    if (d->refi[ip] != d->refi[iq]) return 1;
    if (iabs(d->mv[2 * ip] - d->mv[2 * iq]) >= 4 || iabs(d->mv[2 * ip + 1] - d->mv[2 * iq + 1]) >= 4) return 1;
    return 0;
}
static void edge_filter(uint8_t *s, int step, int bS, int qpav, int chroma, int offA, int offB) {
    int iA = iclip(0, 51, qpav + offA), iB = iclip(0, 51, qpav + offB);
    int a = Alpha[iA], bt = Beta[iB];
    int p0 = s[-step], p1 = s[-2 * step], q0 = s[0], q1 = s[step];
    if (!(bS && iabs(p0 - q0) < a && iabs(p1 - p0) < bt && iabs(q1 - q0) < bt)) return;
    if (bS < 4) {
        int tc0 = Tc0[iA][bS - 1], tc;
        if (chroma) tc = tc0 + 1;
        else {
            int p2 = s[-3 * step], q2 = s[2 * step];
            int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
            tc = tc0 + (ap < bt) + (aq < bt);
            if (ap < bt) s[-2 * step] = (uint8_t)(p1 + iclip(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - 2 * p1) >> 1));
            if (aq < bt) s[step] = (uint8_t)(q1 + iclip(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - 2 * q1) >> 1));
        }
        int dl = iclip(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);
        s[-step] = (uint8_t)clip255(p0 + dl);
        s[0] = (uint8_t)clip255(q0 - dl);
    } else if (chroma) {
        s[-step] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
        s[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
    } else {
        int p2 = s[-3 * step], q2 = s[2 * step], p3 = s[-4 * step], q3 = s[3 * step];
        int ap = iabs(p2 - p0), aq = iabs(q2 - q0), sm = iabs(p0 - q0) < ((a >> 2) + 2);
        if (ap < bt && sm) {
            s[-step] = (uint8_t)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
            s[-2 * step] = (uint8_t)((p2 + p1 + p0 + q0 + 2) >> 2);
            s[-3 * step] = (uint8_t)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
        } else s[-step] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
        if (aq < bt && sm) {
            s[0] = (uint8_t)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
            s[step] = (uint8_t)((p0 + q0 + q1 + q2 + 2) >> 2);
            s[2 * step] = (uint8_t)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
        } else s[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
    }
}
static void deblock(jmo_dec *d) {
    if (d->dis_dbf == 1) return;
    int W = d->W, Wc = W / 2;
    for (int my = 0; my < d->mbh; my++)
        for (int mx = 0; mx < d->mbw; mx++) {
            int qq = d->mi[my * d->mbw + mx].qp;
            for (int vert = 1; vert >= 0; vert--) {
                for (int e = 0; e < 16; e += 4) {
                    if ((e & 4) && d->mi[my * d->mbw + mx].t8) continue;   /* no 4x4 luma edges */
                    if (e == 0 && ((vert && mx == 0) || (!vert && my == 0))) continue;
                    int qp_ = d->mi[vert ? my * d->mbw + mx - (e == 0) : (my - (e == 0)) * d->mbw + mx].qp;
                    int qav = (qp_ + qq + 1) >> 1;
                    int qcav = (QPCt[iclip(0, 51, qp_ + d->cqp_off)] + QPCt[iclip(0, 51, qq + d->cqp_off)] + 1) >> 1;
                    for (int k = 0; k < 16; k++) {
                        int xq = vert ? 16 * mx + e : 16 * mx + k, yq = vert ? 16 * my + k : 16 * my + e;
                        int bS = bs_of(d, vert ? xq - 1 : xq, vert ? yq : yq - 1, xq, yq, e == 0);
                        edge_filter(d->cur[0] + yq * W + xq, vert ? 1 : W, bS, qav, 0, d->offA, d->offB);
                        if ((e & 7) == 0 && (k & 1) == 0) {
                            int cx = vert ? 8 * mx + e / 2 : 8 * mx + k / 2, cy = vert ? 8 * my + k / 2 : 8 * my + e / 2;
                            for (int c = 1; c <= 2; c++) {
                                edge_filter(d->cur[c] + cy * Wc + cx, vert ? 1 : Wc, bS, qcav, 1, d->offA, d->offB);
                            }
                        }
                    }
                }
            }
        }
}

/* chroma lines: in 4:2:0 chroma sample k along an edge maps to luma sample 2k (bS of luma
 * 4x4 edge segment k/2); the loop above filters chroma line k/2 when visiting luma line k (even)
 * using the bS of luma line k, which lies in the same 4-sample segment as 2*(k/2). */

/* more_rbsp_data() (7.2): bits remain before the rbsp_stop_one_bit */
static int more_rbsp_data(const br_t *b) {
    long n = b->n;
    while (n > 0 && b->p[n - 1] == 0) n--;
    if (n == 0) return 0;
    int v = b->p[n - 1], k = 0;
    while (!(v & 1)) { v >>= 1; k++; }
    return b->pos < n * 8 - 1 - k;
}

/* one slice (7.3.3 / 7.3.4).  *pic_done = 1 when it completes the picture (then deblocked). */
static int decode_slice(jmo_dec *d, br_t *b, int nal_type, int nal_ref_idc, int *pic_done) {
    int nmb = d->mbw * d->mbh;
    int first = rue(b);                       /* first_mb_in_slice */
    if (first >= nmb) FAIL("first_mb_in_slice %d", first);
    if (first == 0) d->mbs_done = 0;
    else if (first != d->mbs_done) FAIL("slice starts at MB %d, expected %d", first, d->mbs_done);
    int st = rue(b) % 5;
    if (st != 0 && st != 2) FAIL("slice type %d unsupported", st);
    rue(b);
    rbits(b, d->log2_fn);
    if (nal_type == 5) rue(b);
    rbits(b, d->log2_poc);
    if (st == 0) {
        if (rb(b)) { d->num_ref_l0 = rue(b) + 1; }
        if (rb(b)) FAIL("reordering unsupported");
    }
    if (nal_ref_idc) { if (nal_type == 5) { rb(b); rb(b); } else if (rb(b)) FAIL("MMCO unsupported"); }
    int qp = d->init_qp + rse(b);
    d->dis_dbf = 0; d->offA = d->offB = 0;
    if (d->dfc_present) {
        d->dis_dbf = rue(b);
        if (d->dis_dbf != 1) { d->offA = 2 * rse(b); d->offB = 2 * rse(b); }
    }
    if (st == 0 && !d->have_ref) FAIL("P slice without reference");
    if (first == 0) memset(d->dec4, 0, (size_t)d->W * d->H / 16);
    d->slice_first = first;
    int a = first, more = 1;
    while (more && a < nmb) {
        if (st == 0) {
            int run = rue(b);
            if (b->err) FAIL("skip run");
            for (int i = 0; i < run && a < nmb; i++, a++) {
                if (decode_mb(d, b, a % d->mbw, a / d->mbw, 1, 0, 1, &qp)) return -1;
            }
            if (run > 0) more = more_rbsp_data(b);
        }
        if (more && a < nmb) {
            int t = rue(b);
            if (b->err) FAIL("mb_type at MB %d", a);
            if (decode_mb(d, b, a % d->mbw, a / d->mbw, st == 0, t, 0, &qp)) return -1;
            a++;
            more = more_rbsp_data(b);
        }
    }
    d->mbs_done = a;
    *pic_done = a >= nmb;
    if (*pic_done) deblock(d);
    return 0;
}

int jmo_decode_annexb(jmo_dec *d, const uint8_t *buf, long len, uint8_t *out, long out_cap, int *width, int *height) {
    long i = 0, nframes = 0;
    uint8_t *rbsp = malloc(len + 16);
    while (i + 3 < len) {
        if (!(buf[i] == 0 && buf[i + 1] == 0 && (buf[i + 2] == 1 || (buf[i + 2] == 0 && i + 3 < len && buf[i + 3] == 1)))) { i++; continue; }
        i += buf[i + 2] == 1 ? 3 : 4;
        long j = i;
        while (j + 2 < len && !(buf[j] == 0 && buf[j + 1] == 0 && (buf[j + 2] == 1 || (buf[j + 2] == 0 && j + 3 < len && buf[j + 3] == 1)))) j++;
        if (j + 2 >= len) j = len;
        long n = 0;
        int zeros = 0;
        for (long k = i + 1; k < j; k++) {
            if (zeros >= 2 && buf[k] == 3) { zeros = 0; continue; }
            rbsp[n++] = buf[k];
            zeros = buf[k] == 0 ? zeros + 1 : 0;
        }
        int nal_type = buf[i] & 31, nal_ref = (buf[i] >> 5) & 3;
        br_t b = {rbsp, n, 0, 0};
        int r = 0;
        if (nal_type == 7) r = parse_sps(d, &b);
        else if (nal_type == 8) r = parse_pps(d, &b);
        else if (nal_type == 1 || nal_type == 5) {
            if (!d->have_sps || !d->have_pps) { snprintf(d->err, sizeof d->err, "slice before SPS/PPS"); r = -1; }
            int pic_done = 0;
            if (!r) r = decode_slice(d, &b, nal_type, nal_ref, &pic_done);
            if (!r && pic_done) {
                int cw = d->W - 2 * (d->crop_l + d->crop_r), ch = d->H - 2 * (d->crop_t + d->crop_b);
                long fs = (long)cw * ch * 3 / 2;
                if ((nframes + 1) * fs > out_cap) { snprintf(d->err, sizeof d->err, "output buffer too small"); r = -1; }
                else {
                    uint8_t *o = out + nframes * fs;
                    for (int y = 0; y < ch; y++) memcpy(o + (long)y * cw, d->cur[0] + (long)(y + 2 * d->crop_t) * d->W + 2 * d->crop_l, cw);
                    for (int c = 1; c <= 2; c++)
                        for (int y = 0; y < ch / 2; y++)
                            memcpy(o + (long)cw * ch + (c - 1) * (long)(cw / 2) * (ch / 2) + (long)y * (cw / 2),
                                   d->cur[c] + (long)(y + d->crop_t) * (d->W / 2) + d->crop_l, cw / 2);
                    nframes++;
                    *width = cw; *height = ch;
                    for (int c = 0; c < 3; c++) { uint8_t *t = d->ref[c]; d->ref[c] = d->cur[c]; d->cur[c] = t; }
                    d->have_ref = 1;
                }
            }
        }
        if (r) { free(rbsp); return r < 0 ? -1 : r; }
        i = j;
    }
    free(rbsp);
    return (int)nframes;
}
