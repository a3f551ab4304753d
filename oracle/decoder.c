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

/* ---- CAVLC tables (same normative tables, decoded by prefix match).  The code lengths and the
   coded_block_pattern mapping are shared with the oracle's RD-rate counter (cavlc_bits.c) ---- */
const uint8_t jmo_ct_len[3][4][17] = {
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
const uint8_t jmo_ctdc_len[4][5] = {{2, 6, 6, 6, 6}, {0, 1, 6, 7, 8}, {0, 0, 3, 7, 8}, {0, 0, 0, 6, 7}};
static const uint8_t ctdc_code[4][5] = {{1, 7, 4, 3, 2}, {0, 1, 6, 3, 3}, {0, 0, 1, 2, 2}, {0, 0, 0, 5, 0}};
const uint8_t jmo_tz_len[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6}, {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},
    {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5}, {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5}, {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6}, {6, 4, 5, 3, 2, 2, 3, 3, 6}, {6, 6, 4, 2, 2, 3, 2, 5}, {5, 5, 3, 2, 2, 2, 4}, {4, 4, 3, 3, 1, 3},
    {4, 4, 2, 1, 3}, {3, 3, 1, 2}, {2, 2, 1}, {1, 1}};
static const uint8_t tz_code[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0}, {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},
    {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0}, {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0}, {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0}, {1, 1, 1, 3, 3, 2, 2, 1, 0}, {1, 0, 1, 3, 2, 1, 1, 1}, {1, 0, 1, 3, 2, 1, 1}, {0, 1, 1, 2, 1, 3},
    {0, 1, 1, 1, 1}, {0, 1, 1, 1}, {0, 1, 1}, {0, 1}};
const uint8_t jmo_tzdc_len[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
static const uint8_t tzdc_code[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
const uint8_t jmo_rb_len[7][15] = {{1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3}, {2, 3, 3, 3, 3, 3, 3},
                                      {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
static const uint8_t rb_code[7][15] = {{1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0}, {3, 0, 1, 3, 2, 5, 4},
                                       {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}};
/* Table 9-4: codeNum -> coded_block_pattern (ChromaArrayType 1) */
const uint8_t jmo_cbp_intra[48] = {47, 31, 15, 0, 23, 27, 29, 30, 7, 11, 13, 14, 39, 43, 45, 46, 16, 3, 5, 10, 12, 19, 21, 26,
                                      28, 35, 37, 42, 44, 1, 2, 4, 8, 17, 18, 20, 24, 6, 9, 22, 25, 32, 33, 34, 36, 40, 38, 41};
const uint8_t jmo_cbp_inter[48] = {0, 16, 1, 2, 4, 8, 32, 3, 5, 10, 12, 15, 47, 7, 11, 13, 14, 6, 9, 31, 35, 37, 42, 44,
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
            for (int c = a; c < 5; c++) if (match(b, ctdc_code[a][c], jmo_ctdc_len[a][c])) { t1 = a; tc = c; break; }
    } else if (nC >= 8) {
        int v = rbits(b, 6);
        if (v == 3) { tc = 0; t1 = 0; } else { tc = (v >> 2) + 1; t1 = v & 3; }
    } else {
        int t = nC < 2 ? 0 : nC < 4 ? 1 : 2;
        for (int a = 0; a < 4 && tc < 0; a++)
            for (int c = a; c < 17; c++) if (c > 0 || a == 0) if (match(b, ct_code[t][a][c], jmo_ct_len[t][a][c])) { t1 = a; tc = c; break; }
    }
    if (tc < 0 || tc > maxn || t1 > tc) return -1;
    if (!tc) return 0;
    int lev[16];
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = 0; i < tc; i++) {
        if (i < t1) { lev[i] = rb(b) ? -1 : 1; continue; }
        int prefix = 0;
        while (!rb(b)) { if (++prefix > 28 || b->err) return -1; }
        int size = (prefix == 14 && sl == 0) ? 4 : (prefix >= 15 ? prefix - 3 : sl);
        int code = (imin(15, prefix) << sl) + (size ? (int)rbits(b, size) : 0);
        if (prefix >= 15 && sl == 0) code += 15;
        if (prefix >= 16) code += (1 << (prefix - 3)) - 4096;   /* 9.2.2.1 */
        if (i == t1 && t1 < 3) code += 2;
        lev[i] = (code & 1) ? (-code - 1) >> 1 : (code + 2) >> 1;
        if (sl == 0) sl = 1;
        if (iabs(lev[i]) > (3 << (sl - 1)) && sl < 6) sl++;
    }
    int tz = 0;
    if (tc < maxn) {
        tz = -1;
        if (nC == -1) { for (int z = 0; z <= 4 - tc; z++) if (match(b, tzdc_code[tc - 1][z], jmo_tzdc_len[tc - 1][z])) { tz = z; break; } }
        else { for (int z = 0; z <= 16 - tc; z++) if (match(b, tz_code[tc - 1][z], jmo_tz_len[tc - 1][z])) { tz = z; break; } }
        if (tz < 0) return -1;
    }
    int zl = tz, run[16];
    for (int i = 0; i < tc - 1; i++) {
        run[i] = 0;
        if (zl > 0) {
            int t = zl > 6 ? 6 : zl - 1, got = -1;
            for (int r = 0; r <= imin(zl, 14); r++) if (match(b, rb_code[t][r], jmo_rb_len[t][r])) { got = r; break; }
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
    /* CABAC context selection state (9.3.3.1.1) */
    int cbp;              /* coded_block_pattern (P_Skip 0)                                 */
    int cmode;            /* intra_chroma_pred_mode                                          */
    int cbf_dc;           /* coded_block_flag: bit 0 luma DC, 1 Cb DC, 2 Cr DC               */
    int cbf4;             /* luma 4x4 blocks (raster)                                        */
    int cbfc[2];          /* chroma AC blocks                                                */
} mbinfo;

typedef struct { br_t *b; uint32_t range, ofs; uint8_t st[JMO_NCTX], mps[JMO_NCTX]; } cabd_t;

struct jmo_dec {
    char err[256];
    int have_sps, have_pps;
    int mbw, mbh, W, H, crop_l, crop_r, crop_t, crop_b;
    int log2_fn, poc_type, log2_poc;
    int num_ref_l0, init_qp, cqp_off, dfc_present, cip, t8mode;
    pel *cur[3], *ref[3];  /* 16-bit samples at every bit depth                               */
    int bd, maxv, qpbd;   /* BitDepthY = BitDepthC, (1 << bd) - 1, QpBdOffset = 6 (bd - 8)   */
    int have_ref;
    mbinfo *mi;
    int16_t *mv;          /* per 4x4 [2] */
    int8_t *refi;         /* per 4x4 */
    int8_t *dec4;         /* per 4x4: decoded in the current picture */
    int dis_dbf, offA, offB;
    int slice_first;      /* first MB of the current slice: MBs before it are unavailable (6.4.8) */
    int mbs_done;         /* MBs of the current picture decoded so far (a picture may have many slices) */
    int cabac;            /* PPS entropy_coding_mode_flag                                    */
    int16_t *mvd;         /* per 4x4 [2]: mvd_l0 (CABAC contexts)                            */
    cabd_t cab;
    int prev_qpd;         /* the previous MB of the slice had mb_qp_delta != 0               */
};

int jmo_dec_create(jmo_dec **out) { *out = (jmo_dec *)calloc(1, sizeof(jmo_dec)); return *out ? 0 : JMH_E_OOM; }
void jmo_dec_destroy(jmo_dec *d) {
    if (!d) return;
    for (int i = 0; i < 3; i++) { free(d->cur[i]); free(d->ref[i]); }
    free(d->mi); free(d->mv); free(d->refi); free(d->dec4); free(d->mvd);
    free(d);
}
const char *jmo_dec_error(const jmo_dec *d) { return d->err; }
int jmo_dec_bit_depth(const jmo_dec *d) { return d->have_sps ? d->bd : 0; }

static void alloc_pics(jmo_dec *d) {
    for (int i = 0; i < 3; i++) { free(d->cur[i]); free(d->ref[i]); }
    size_t ls = (size_t)d->W * d->H;
    d->cur[0] = calloc(ls, sizeof(pel)); d->cur[1] = calloc(ls / 4, sizeof(pel)); d->cur[2] = calloc(ls / 4, sizeof(pel));
    d->ref[0] = calloc(ls, sizeof(pel)); d->ref[1] = calloc(ls / 4, sizeof(pel)); d->ref[2] = calloc(ls / 4, sizeof(pel));
    free(d->mi); free(d->mv); free(d->refi); free(d->dec4); free(d->mvd);
    d->mi = calloc((size_t)d->mbw * d->mbh, sizeof(mbinfo));
    d->mvd = calloc(ls / 16 * 2, sizeof(int16_t));
    d->mv = calloc(ls / 16 * 2, sizeof(int16_t));
    d->refi = calloc(ls / 16, 1);
    d->dec4 = calloc(ls / 16, 1);
    d->have_ref = 0;
}

static int parse_sps(jmo_dec *d, br_t *b) {
    int profile = rbits(b, 8);
    rbits(b, 16);
    rue(b);
    d->bd = 8;
    if (profile == 100 || profile == 110) {   /* High / High 10: 4:2:0, BitDepthC = BitDepthY, flat scaling lists */
        int cf = rue(b), bdl = rue(b) + 8, bdc = rue(b) + 8;
        if (cf != 1 || bdl != bdc || bdl > (profile == 110 ? 10 : 8) || rb(b) || rb(b)) {
            snprintf(d->err, sizeof d->err, "High profile SPS options unsupported");
            return -1;
        }
        d->bd = bdl;
    } else if (profile >= 100) { snprintf(d->err, sizeof d->err, "profile %d unsupported", profile); return -1; }
    d->maxv = (1 << d->bd) - 1;
    d->qpbd = 6 * (d->bd - 8);
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
    d->cabac = rb(b);                     /* entropy_coding_mode_flag */
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
/* ... for Intra prediction: with constrained_intra_pred_flag an inter (or skipped) neighbour's
 * samples are not available (8.3.1.2, 8.3.2.2, 8.3.3, 8.3.4) */
static int iavail_mb(const jmo_dec *d, int mx, int my, int cmx, int cmy) {
    if (!avail_mb(d, mx, my, cmx, cmy)) return 0;
    const int t = d->mi[my * d->mbw + mx].mbtype;
    return !d->cip || t == 1 || t == 2 || t == 4;
}
/* availability of luma sample at MB-relative (x,y) for intra 4x4 block at (bx,by) */
static int lavail(const jmo_dec *d, int mx, int my, int x, int y, int blk_idx) {
    if (x > 15 || y > 15) { if (x > 15 && y < 0) return iavail_mb(d, mx + 1, my - 1, mx, my); return 0; }
    if (x < 0 && y < 0) return iavail_mb(d, mx - 1, my - 1, mx, my);
    if (x < 0) return iavail_mb(d, mx - 1, my, mx, my);
    if (y < 0) return iavail_mb(d, mx, my - 1, mx, my);
    (void)blk_idx;
    return 1;
}
static void pred4x4(const jmo_dec *d, int mx, int my, int bx, int by, int blk_idx, int mode, pel *pr, int *ok) {
    const pel *R = d->cur[0];
    int W = d->W, X = 16 * mx + bx, Y = 16 * my + by;
    int up = lavail(d, mx, my, bx, by - 1, blk_idx), left = lavail(d, mx, my, bx - 1, by, blk_idx);
    int ul = lavail(d, mx, my, bx - 1, by - 1, blk_idx);
    int ur = lavail(d, mx, my, bx + 4, by - 1, blk_idx);
    if (blk_idx == 3 || blk_idx == 11 || blk_idx == 7 || blk_idx == 13 || blk_idx == 15) ur = 0;
    if ((blk_idx == 5) && !iavail_mb(d, mx + 1, my - 1, mx, my)) ur = 0;
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
                else v = 1 << (d->bd - 1);
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
            pr[4 * y + x] = (pel)v;
        }
#undef T
#undef L
}
static int pred16(const jmo_dec *d, int mx, int my, int mode, pel *pr) {
    const pel *R = d->cur[0];
    int W = d->W, X = 16 * mx, Y = 16 * my;
    int up = iavail_mb(d, mx, my - 1, mx, my), left = iavail_mb(d, mx - 1, my, mx, my), ul = iavail_mb(d, mx - 1, my - 1, mx, my);
    int T[17], L[17];                   /* index 0 = corner */
    T[0] = L[0] = ul ? R[(Y - 1) * W + X - 1] : 0;
    for (int i = 0; i < 16; i++) { T[1 + i] = up ? R[(Y - 1) * W + X + i] : 0; L[1 + i] = left ? R[(Y + i) * W + X - 1] : 0; }
    if (mode == 0 && !up) return -1;
    if (mode == 1 && !left) return -1;
    if (mode == 3 && !(up && left && ul)) return -1;
    int st = 0, sl = 0;
    for (int i = 1; i <= 16; i++) { st += T[i]; sl += L[i]; }
    int dc = (up && left) ? (st + sl + 16) >> 5 : up ? (st + 8) >> 4 : left ? (sl + 8) >> 4 : 1 << (d->bd - 1);
    int H = 0, V = 0;
    for (int xp = 0; xp < 8; xp++) { H += (xp + 1) * (T[1 + 8 + xp] - T[1 + 6 - xp]); V += (xp + 1) * (L[1 + 8 + xp] - L[1 + 6 - xp]); }
    int a = 16 * (L[16] + T[16]), bb = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) {
            int v = mode == 0 ? T[1 + x] : mode == 1 ? L[1 + y] : mode == 2 ? dc : iclip(0, d->maxv, (a + bb * (x - 7) + c * (y - 7) + 16) >> 5);
            pr[16 * y + x] = (pel)v;
        }
    return 0;
}
static int predc(const jmo_dec *d, int mx, int my, int comp, int mode, pel *pr) {
    const pel *R = d->cur[comp];
    const int dcd = 1 << (d->bd - 1);
    int W = d->W / 2, X = 8 * mx, Y = 8 * my;
    int up = iavail_mb(d, mx, my - 1, mx, my), left = iavail_mb(d, mx - 1, my, mx, my), ul = iavail_mb(d, mx - 1, my - 1, mx, my);
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
            if ((xo == 0 && yo == 0) || (xo > 0 && yo > 0)) v = (up && left) ? (su + sv + 4) >> 3 : left ? (sv + 2) >> 2 : up ? (su + 2) >> 2 : dcd;
            else if (xo > 0) v = up ? (su + 2) >> 2 : left ? (sv + 2) >> 2 : dcd;
            else v = left ? (sv + 2) >> 2 : up ? (su + 2) >> 2 : dcd;
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
                    w = iclip(0, d->maxv, (a + bb * (xx - 3) + c * (yy - 3) + 16) >> 5);
                }
                pr[8 * yy + xx] = (pel)w;
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
static void recon4x4(int32_t *c, const pel *pred, int ps, pel *out, int os, int maxv) {
    int32_t r[16];
    jmo_inverse4x4(c, r);
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) out[y * os + x] = (pel)iclip(0, maxv, pred[y * ps + x] + ((r[4 * y + x] + 32) >> 6));
}

/* ---- Intra_8x8 (8.3.2.2): the 25 reference samples as one edge e[0..24] running from
 * p[-1,7] up to p[-1,0] (e[7-y]), the corner p[-1,-1] (e[8]) and along p[0..15,-1] (e[9+x]);
 * the 8.3.2.2.1 filter is a [1 2 1] tap along the edge whose missing outer neighbour is
 * replaced by the centre sample, and every directional mode reads that filtered edge. */
static int pred8x8(const jmo_dec *d, int mx, int my, int b8, int mode, pel *pr) {
    const pel *R = d->cur[0];
    int W = d->W, bx = 8 * (b8 & 1), by = 8 * (b8 >> 1), X = 16 * mx + bx, Y = 16 * my + by;
    int left = bx ? 1 : iavail_mb(d, mx - 1, my, mx, my);
    int up = by ? 1 : iavail_mb(d, mx, my - 1, mx, my);
    int ul = bx && by ? 1 : bx ? iavail_mb(d, mx, my - 1, mx, my) : by ? iavail_mb(d, mx - 1, my, mx, my) : iavail_mb(d, mx - 1, my - 1, mx, my);
    int ur = b8 == 0 ? iavail_mb(d, mx, my - 1, mx, my) : b8 == 1 ? iavail_mb(d, mx + 1, my - 1, mx, my) : b8 == 2;
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
    int dc = 1 << (d->bd - 1), st = 0, sl = 0;
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
            pr[8 * y + x] = (pel)v;
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
static void recon8x8(const int *c64, int qp, const pel *pred, int ps, pel *out, int os, int maxv) {
    int32_t m[64], r[64];
    for (int k = 0; k < 64; k++) {
        int x = zz8[k][0], y = zz8[k][1], ls = lscale8(qp % 6, y, x), c = c64[k];
        m[8 * y + x] = qp >= 36 ? c * ls * (1 << (qp / 6 - 6)) : (c * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
    jmo_inverse8x8(m, r);
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) out[y * os + x] = (pel)iclip(0, maxv, pred[y * ps + x] + ((r[8 * y + x] + 32) >> 6));
}

/* ---- inter prediction (8.4.2.2) ------------------------------------------------------- */
static void inter_pred(const jmo_dec *d, int mx, int my, const int16_t mv16[16][2], pel *py, pel *pu, pel *pv) {
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) {
            const int16_t *v = mv16[(y >> 2) * 4 + (x >> 2)];
            py[16 * y + x] = (pel)jmo_qpel_px(d->ref[0], d->W, d->H, d->W, 4 * (16 * mx + x) + v[0], 4 * (16 * my + y) + v[1], d->maxv);
        }
    int Wc = d->W / 2, Hc = d->H / 2;
    for (int c = 1; c <= 2; c++)
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) {
                const int16_t *v = mv16[(y >> 1) * 4 + (x >> 1)];
                int xi = 8 * mx + x + (v[0] >> 3), yi = 8 * my + y + (v[1] >> 3), fx = v[0] & 7, fy = v[1] & 7;
                const pel *R = d->ref[c];
                int A = R[iclip(0, Hc - 1, yi) * Wc + iclip(0, Wc - 1, xi)], B = R[iclip(0, Hc - 1, yi) * Wc + iclip(0, Wc - 1, xi + 1)];
                int C = R[iclip(0, Hc - 1, yi + 1) * Wc + iclip(0, Wc - 1, xi)], D = R[iclip(0, Hc - 1, yi + 1) * Wc + iclip(0, Wc - 1, xi + 1)];
                (c == 1 ? pu : pv)[8 * y + x] = (pel)(((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6);
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

/* ---- one macroblock's syntax, parsed by CAVLC (9.2) or CABAC (9.3), then reconstructed ---- */
typedef struct {
    int skip;              /* P_Skip                                                          */
    int intra_type;        /* -1 inter (or P_Skip), 0 I_NxN, 1 I_16x16                         */
    int i16mode, cmode, cbp;
    int ipm[16];           /* Intra4x4 / Intra8x8 modes per 4x4 (raster)                       */
    int16_t mv16[16][2];
    int dc16[16];          /* Intra16x16DCLevel (scan order)                                   */
    int l4[16][16];        /* per 4x4 (raster): levels in zig-zag order (I16: AC at 1..15)      */
    int l8[4][64];         /* per 8x8: 8x8 zig-zag order                                        */
    int cdc[2][4];         /* chroma DC c0..c3                                                  */
    int cac[2][4][16];     /* chroma AC (zig-zag, [0] unused)                                   */
} mbsyn;

/* reset the MB's partition / motion state before parsing it */
static void mb_begin(jmo_dec *d, int mx, int my, mbsyn *s) {
    memset(&d->mi[my * d->mbw + mx], 0, sizeof(mbinfo));
    memset(s, 0, sizeof(*s));
    int W4 = d->W / 4;
    for (int k = 0; k < 16; k++) {
        int i = (4 * my + (k >> 2)) * W4 + 4 * mx + (k & 3);
        d->dec4[i] = 0; d->refi[i] = -1; d->mv[2 * i] = d->mv[2 * i + 1] = 0;
        d->mvd[2 * i] = d->mvd[2 * i + 1] = 0;
    }
}

/* P_Skip motion (8.4.1.1) */
static void skip_motion(jmo_dec *d, int mx, int my, mbsyn *s) {
    int ia = 0, ib = 0;
    int aa = nb4(d, mx, my, -1, 0, &ia), ab = nb4(d, mx, my, 0, -1, &ib);
    int mvx = 0, mvy = 0;
    if (aa && ab && !(d->refi[ia] == 0 && !d->mv[2 * ia] && !d->mv[2 * ia + 1]) && !(d->refi[ib] == 0 && !d->mv[2 * ib] && !d->mv[2 * ib + 1])) {
        int p[2];
        mvpred(d, mx, my, 0, 0, 16, 16, 0, p);
        mvx = p[0]; mvy = p[1];
    }
    set_part(d, mx, my, 0, 0, 16, 16, mvx, mvy, 0, s->mv16);
    s->skip = 1;
    s->intra_type = -1;
    d->mi[my * d->mbw + mx].mbtype = 3;
}

/* predIntra4x4PredMode / predIntra8x8PredMode (8.3.1.1 / 8.3.2.1); ipm: this MB's modes so far */
static int pred_ipm(const jmo_dec *d, int mx, int my, int x4, int y4, const int *ipm) {
    int ma, mb;
    /* dcPredModePredictedFlag: a neighbour not available, or inter under constrained_intra_pred */
    if (x4 > 0) ma = ipm[y4 * 4 + x4 - 1];
    else if (iavail_mb(d, mx - 1, my, mx, my)) { const mbinfo *n = &d->mi[my * d->mbw + mx - 1]; ma = (n->mbtype == 1 || n->mbtype == 4) ? n->ipm[y4 * 4 + 3] : 2; }
    else return 2;
    if (y4 > 0) mb = ipm[(y4 - 1) * 4 + x4];
    else if (iavail_mb(d, mx, my - 1, mx, my)) { const mbinfo *n = &d->mi[(my - 1) * d->mbw + mx]; mb = (n->mbtype == 1 || n->mbtype == 4) ? n->ipm[12 + x4] : 2; }
    else return 2;
    return imin(ma, mb);
}
/* the intra mode of 4x4 block (x4, y4), 8x8 blocks fill their four 4x4 */
static void set_ipm(mbsyn *s, int x4, int y4, int mode, int t8) {
    if (!t8) { s->ipm[y4 * 4 + x4] = mode; return; }
    for (int k = 0; k < 4; k++) s->ipm[(y4 + (k >> 1)) * 4 + x4 + (k & 1)] = mode;
}

static int parse_cavlc(jmo_dec *d, br_t *b, int mx, int my, int slice_p, int t, mbsyn *s, int *qp) {
    mbinfo *mi = &d->mi[my * d->mbw + mx];
    int intra_type = -1, no_sub8x8 = 0, cbp = 0;
    if (slice_p) { if (t >= 5) { t -= 5; intra_type = t == 0 ? 0 : 1; } }
    else intra_type = t == 0 ? 0 : 1;
    s->intra_type = intra_type;
    if (intra_type == 1) {
        if (t > 24) FAIL("I_PCM unsupported");
        s->i16mode = (t - 1) % 4;
        cbp = (((t - 1) / 4) % 3) << 4 | ((t >= 13) ? 15 : 0);
    }
    if (intra_type >= 0) {
        mi->intra = 1;
        mi->mbtype = intra_type == 0 ? 1 : 2;
        if (intra_type == 0 && d->t8mode) mi->t8 = rb(b);
        if (intra_type == 0) {
            if (mi->t8) mi->mbtype = 4;
            for (int blk = 0; blk < 16; blk += mi->t8 ? 4 : 1) {
                int x4 = ((blk >> 2) & 1) * 2 + (blk & 1), y4 = (blk >> 3) * 2 + ((blk >> 1) & 1);
                int flag = rb(b), rem = flag ? 0 : (int)rbits(b, 3);
                int pm = pred_ipm(d, mx, my, x4, y4, s->ipm);
                set_ipm(s, x4, y4, flag ? pm : (rem < pm ? rem : rem + 1), mi->t8);
            }
            for (int k = 0; k < 16; k++) mi->ipm[k] = (int8_t)s->ipm[k];
        }
        s->cmode = rue(b);
        if (s->cmode > 3) FAIL("bad chroma mode");
    } else {
        mi->mbtype = 0;
        if (t > 4) FAIL("bad P mb_type %d", t);
        if (d->num_ref_l0 > 1) FAIL("multiple refs unsupported");
        no_sub8x8 = 1;
        if (t == 3 || t == 4) {
            int sub[4];
            for (int i = 0; i < 4; i++) { sub[i] = rue(b); if (sub[i] > 3) FAIL("bad sub_mb_type"); if (sub[i]) no_sub8x8 = 0; }
            for (int i = 0; i < 4; i++) {
                int ox = (i & 1) * 8, oy = (i >> 1) * 8;
                int sw = sub[i] == 0 || sub[i] == 1 ? 8 : 4, sh = sub[i] == 0 || sub[i] == 2 ? 8 : 4;
                for (int y = 0; y < 8; y += sh)
                    for (int x = 0; x < 8; x += sw) {
                        int p[2];
                        mvpred(d, mx, my, ox + x, oy + y, sw, sh, 0, p);
                        int dx = rse(b), dy = rse(b);
                        set_part(d, mx, my, ox + x, oy + y, sw, sh, p[0] + dx, p[1] + dy, 0, s->mv16);
                    }
            }
        } else {
            int np = t == 0 ? 1 : 2, w = t == 2 ? 8 : 16, h = t == 1 ? 8 : 16;
            for (int pi = 0; pi < np; pi++) {
                int x = t == 2 ? 8 * pi : 0, y = t == 1 ? 8 * pi : 0, p[2];
                mvpred(d, mx, my, x, y, w, h, 0, p);
                int dx = rse(b), dy = rse(b);
                set_part(d, mx, my, x, y, w, h, p[0] + dx, p[1] + dy, 0, s->mv16);
            }
        }
    }
    if (intra_type != 1) {
        int code = rue(b);
        if (code > 47) FAIL("bad cbp code");
        cbp = intra_type == 0 ? jmo_cbp_intra[code] : jmo_cbp_inter[code];
        if (intra_type < 0 && (cbp & 15) && d->t8mode && no_sub8x8) mi->t8 = rb(b);
    }
    s->cbp = cbp;
    if (cbp > 0 || intra_type == 1) {
        int dq = rse(b);
        *qp = (*qp + dq + 52 + 2 * d->qpbd) % (52 + d->qpbd) - d->qpbd;   /* 7-37 */
    }
    /* residual (7.3.5.3, CAVLC): I16 DC, luma, chroma DC Cb Cr, chroma AC Cb Cr */
    int cbpl = cbp & 15, cbpc = cbp >> 4;
    if (intra_type == 1 && read_block(b, calc_nc(d, mx, my, 0, 0, 0, mi->tc), 16, s->dc16) < 0) FAIL("I16 DC at %d,%d", mx, my);
    for (int b8 = 0; b8 < 4; b8++)
        for (int i4 = 0; i4 < 4; i4++) {
            int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1), c[16] = {0}, tc = 0;
            if (cbpl & (1 << b8)) {
                int nC = calc_nc(d, mx, my, 0, x4, y4, mi->tc);
                if (intra_type == 1) { tc = read_block(b, nC, 15, c + 1); }
                else tc = read_block(b, nC, 16, c);
                if (tc < 0) FAIL("luma block %d at MB %d,%d", b8 * 4 + i4, mx, my);
            }
            mi->tc[y4 * 4 + x4] = (uint8_t)tc;
            if (mi->t8) for (int k = 0; k < 16; k++) s->l8[b8][4 * k + i4] = c[k];   /* 4 interleaved blocks */
            else for (int k = 0; k < 16; k++) s->l4[y4 * 4 + x4][k] = c[k];
        }
    if (cbpc)
        for (int comp = 0; comp < 2; comp++) if (read_block(b, -1, 4, s->cdc[comp]) < 0) FAIL("chroma DC");
    if (cbpc == 2)
        for (int comp = 0; comp < 2; comp++)
            for (int k = 0; k < 4; k++) {
                int tc = read_block(b, calc_nc(d, mx, my, 1 + comp, k & 1, k >> 1, mi->tc), 15, s->cac[comp][k] + 1);
                if (tc < 0) FAIL("chroma AC");
                mi->tc[16 + 4 * comp + k] = (uint8_t)tc;
            }
    return b->err ? -1 : 0;
}

/* ---- CABAC parsing (9.3): arithmetic decoding engine, initialisation, binarisations ----- */
/* Table 9-44 (own copy; the encoder's is in host/cabac.c).  Shared with the oracle's RD-rate
   encoder (cabac_enc.c), which has no other tie to this decoder */
const uint8_t jmo_lps_range[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205}, {116, 142, 169, 195}, {111, 135, 160, 185},
    {105, 128, 152, 175}, {100, 122, 144, 166}, {95, 116, 137, 158},  {90, 110, 130, 150},  {85, 104, 123, 142},  {81, 99, 117, 135},
    {77, 94, 111, 128},   {73, 89, 105, 122},   {69, 85, 100, 116},   {66, 80, 95, 110},    {62, 76, 90, 104},    {59, 72, 86, 99},
    {56, 69, 81, 94},     {53, 65, 77, 89},     {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},
    {41, 50, 59, 69},     {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},     {33, 41, 48, 56},     {32, 39, 46, 53},
    {30, 37, 43, 50},     {29, 35, 41, 48},     {27, 33, 39, 45},     {26, 31, 37, 43},     {24, 30, 35, 41},     {23, 28, 33, 39},
    {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},     {19, 23, 27, 31},     {18, 22, 26, 30},     {17, 21, 25, 28},
    {16, 20, 23, 27},     {15, 19, 22, 25},     {14, 18, 21, 24},     {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},
    {12, 14, 17, 20},     {11, 14, 16, 19},     {11, 13, 15, 18},     {10, 12, 15, 17},     {10, 12, 14, 16},     {9, 11, 13, 15},
    {9, 11, 12, 14},      {8, 10, 12, 14},      {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},       {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2}};
const uint8_t jmo_lps_next[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12, 13, 13, 15, 15, 16, 16,
                                     18, 18, 19, 19, 21, 21, 22, 22, 23, 24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30,
                                     31, 32, 32, 33, 33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};
/* Tables 9-12 .. 9-33 as runs of consecutive ctxIdx: {first ctxIdx, count} then (m, n) pairs;
   I slices and cabac_init_idc 0 (own copy, typed per syntax element) */
static const int16_t ctxinit_I[] = {
    0, 11, 20, -15, 2, 54, 3, 74, 20, -15, 2, 54, 3, 74, -28, 127, -23, 104, -6, 53, -1, 54, 7, 51,
    60, 4, 0, 41, 0, 63, 0, 63, 0, 63,                                               /* mb_qp_delta        */
    64, 4, -9, 83, 4, 86, 0, 97, -7, 72,                                             /* intra chroma mode   */
    68, 2, 13, 41, 3, 62,                                                            /* intra pred modes    */
    73, 4, -17, 127, -13, 102, 0, 82, -7, 74,                                        /* cbp luma            */
    77, 8, -21, 107, -27, 127, -31, 127, -24, 127, -18, 95, -27, 127, -21, 114, -30, 127,   /* cbp chroma */
    85, 20, -17, 123, -12, 115, -16, 122, -11, 115, -12, 63, -2, 68, -15, 84, -13, 104, -3, 70, -8, 93,
            -10, 90, -30, 127, -1, 74, -6, 97, -7, 91, -20, 127, -4, 56, -5, 82, -7, 76, -22, 125,   /* cbf */
    105, 61, -7, 93, -11, 87, -3, 77, -5, 71, -4, 63, -4, 68, -12, 84, -7, 62, -7, 65, 8, 61, 5, 56, -2, 66, 1, 64,
             0, 61, -2, 78, 1, 50, 7, 52, 10, 35, 0, 44, 11, 38, 1, 45, 0, 46, 5, 44, 31, 17, 1, 51, 7, 50, 28, 19,
             16, 33, 14, 62, -13, 108, -15, 100, -13, 101, -13, 91, -12, 94, -10, 88, -16, 84, -10, 86, -7, 83,
             -13, 87, -19, 94, 1, 70, 0, 72, -5, 74, 18, 59, -8, 102, -15, 100, 0, 95, -4, 75, 2, 72, -11, 75,
             -3, 71, 15, 46, -13, 69, 0, 62, 0, 65, 21, 37, -15, 72, 9, 57, 16, 54, 0, 62, 12, 72,       /* sig */
    166, 61, 24, 0, 15, 9, 8, 25, 13, 18, 15, 9, 13, 19, 10, 37, 12, 18, 6, 29, 20, 33, 15, 30, 4, 45, 1, 58,
             0, 62, 7, 61, 12, 38, 11, 45, 15, 39, 11, 42, 13, 44, 16, 45, 12, 41, 10, 49, 30, 34, 18, 42, 10, 55,
             17, 51, 17, 46, 0, 89, 26, -19, 22, -17, 26, -17, 30, -25, 28, -20, 33, -23, 37, -27, 33, -23,
             40, -28, 38, -17, 33, -11, 40, -15, 41, -6, 38, 1, 41, 17, 30, -6, 27, 3, 26, 22, 37, -16, 35, -4,
             38, -8, 38, -3, 37, 3, 38, 5, 42, 0, 35, 16, 39, 22, 14, 48, 27, 37, 21, 60, 12, 68, 2, 97, /* last */
    227, 49, -3, 71, -6, 42, -5, 50, -3, 54, -2, 62, 0, 58, 1, 63, -2, 72, -1, 74, -9, 91, -5, 67, -5, 27,
             -3, 39, -2, 44, 0, 46, -16, 64, -8, 68, -10, 78, -6, 77, -10, 86, -12, 92, -15, 55, -10, 60, -6, 62,
             -4, 65, -12, 73, -8, 76, -7, 80, -9, 88, -17, 110, -11, 97, -20, 84, -11, 79, -6, 73, -4, 74,
             -13, 86, -13, 96, -11, 97, -19, 117, -8, 78, -5, 33, -4, 48, -2, 53, -3, 62, -13, 71, -10, 79,
             -12, 86, -13, 90, -14, 97,                                                            /* levels */
    399, 3, 31, 21, 31, 31, 25, 50,                                                  /* transform_size_8x8  */
    402, 15, -17, 120, -20, 112, -18, 114, -11, 85, -15, 92, -14, 89, -26, 71, -15, 81, -14, 80, 0, 68,
             -14, 70, -24, 56, -23, 68, -24, 50, -11, 74,
    417, 9, 23, -13, 26, -13, 40, -15, 49, -14, 44, 3, 45, 6, 44, 34, 33, 54, 19, 82,
    426, 10, -3, 75, -1, 23, 1, 34, 1, 43, 0, 54, -2, 55, 0, 61, 1, 64, 0, 68, -9, 92,
    -1};
static const int16_t ctxinit_P0[] = {
    0, 11, 20, -15, 2, 54, 3, 74, 20, -15, 2, 54, 3, 74, -28, 127, -23, 104, -6, 53, -1, 54, 7, 51,
    11, 3, 23, 33, 23, 2, 21, 0,                                                     /* mb_skip_flag        */
    14, 7, 1, 9, 0, 49, -37, 118, 5, 57, -13, 78, -11, 65, 1, 62,                    /* mb_type P           */
    21, 3, 12, 49, -4, 73, 17, 50,                                                   /* sub_mb_type         */
    40, 7, -3, 69, -6, 81, -11, 96, 6, 55, 7, 67, -5, 86, 2, 88,                     /* mvd x               */
    47, 7, 0, 58, -3, 76, -10, 94, 5, 54, 4, 69, -3, 81, 0, 88,                      /* mvd y               */
    54, 6, -7, 67, -5, 74, -4, 74, -5, 80, -7, 72, 1, 58,                            /* ref_idx             */
    60, 4, 0, 41, 0, 63, 0, 63, 0, 63,
    64, 4, -9, 83, 4, 86, 0, 97, -7, 72,
    68, 2, 13, 41, 3, 62,
    73, 4, -27, 126, -28, 98, -25, 101, -23, 67,
    77, 8, -28, 82, -20, 94, -16, 83, -22, 110, -21, 91, -18, 102, -13, 93, -29, 127,
    85, 20, -7, 92, -5, 89, -7, 96, -13, 108, -3, 46, -1, 65, -1, 57, -9, 93, -3, 74, -9, 92,
            -8, 87, -23, 126, 5, 54, 6, 60, 6, 59, 6, 69, -1, 48, 0, 68, -4, 69, -8, 88,
    105, 61, -2, 85, -6, 78, -1, 75, -7, 77, 2, 54, 5, 50, -3, 68, 1, 50, 6, 42, -4, 81, 1, 63, -4, 70, 0, 67,
             2, 57, -2, 76, 11, 35, 4, 64, 1, 61, 11, 35, 18, 25, 12, 24, 13, 29, 13, 36, -10, 93, -7, 73,
             -2, 73, 13, 46, 9, 49, -7, 100, 9, 53, 2, 53, 5, 53, -2, 61, 0, 56, 0, 56, -13, 63, -5, 60,
             -1, 62, 4, 57, -6, 69, 4, 57, 14, 39, 4, 51, 13, 68, 3, 64, 1, 61, 9, 63, 7, 50, 16, 39, 5, 44,
             4, 52, 11, 48, -5, 60, -1, 59, 0, 59, 22, 33, 5, 44, 14, 43, -1, 78, 0, 60, 9, 69,
    166, 61, 11, 28, 2, 40, 3, 44, 0, 49, 0, 46, 2, 44, 2, 51, 0, 47, 4, 39, 2, 62, 6, 46, 0, 54, 3, 54,
             2, 58, 4, 63, 6, 51, 6, 57, 7, 53, 6, 52, 6, 55, 11, 45, 14, 36, 8, 53, -1, 82, 7, 55, -3, 78,
             15, 46, 22, 31, -1, 84, 25, 7, 30, -7, 28, 3, 28, 4, 32, 0, 34, -1, 30, 6, 30, 6, 32, 9, 31, 19,
             26, 27, 26, 30, 37, 20, 28, 34, 17, 70, 1, 67, 5, 59, 9, 67, 16, 30, 18, 32, 18, 35, 22, 29,
             24, 31, 23, 38, 18, 43, 20, 41, 11, 63, 9, 59, 9, 64, -1, 94, -2, 89, -9, 108,
    227, 49, -6, 76, -2, 44, 0, 45, 0, 52, -3, 64, -2, 59, -4, 70, -4, 75, -8, 82, -17, 102, -9, 77, 3, 24,
             0, 42, 0, 48, 0, 55, -6, 59, -7, 71, -12, 83, -11, 87, -30, 119, 1, 58, -3, 29, -1, 36, 1, 38,
             2, 43, -6, 55, 0, 58, 0, 64, -3, 74, -10, 90, 0, 70, -4, 29, 5, 31, 7, 42, 1, 59, -2, 58,
             -3, 72, -3, 81, -11, 97, 0, 58, 8, 5, 10, 14, 14, 18, 13, 27, 2, 40, 0, 58, -3, 70, -6, 79, -8, 85,
    399, 3, 12, 40, 11, 51, 14, 59,
    402, 15, -4, 79, -7, 71, -5, 69, -9, 70, -8, 66, -10, 68, -19, 73, -12, 69, -16, 70, -15, 67, -20, 62,
             -19, 70, -16, 66, -22, 65, -20, 63,
    417, 9, 9, -2, 26, -9, 33, -9, 39, -7, 41, -2, 45, 3, 49, 9, 45, 27, 36, 59,
    426, 10, -6, 66, -7, 35, -7, 42, -8, 45, -5, 48, -12, 56, -6, 60, -5, 62, -8, 66, -8, 76,
    -1};

/* 9.3.1.1: every context this codec uses (spec ctxIdx, < JMO_NCTX) for an I slice or cabac_init_idc 0 */
void jmo_cabac_init_models(int slice_i, int qp, uint8_t *st, uint8_t *mps) {
    const int16_t *t = slice_i ? ctxinit_I : ctxinit_P0;
    memset(st, 0, JMO_NCTX);
    memset(mps, 0, JMO_NCTX);
    while (*t >= 0) {
        int first = t[0], cnt = t[1];
        t += 2;
        for (int i = 0; i < cnt; i++, t += 2) {
            int pre = iclip(1, 126, ((t[0] * iclip(0, 51, qp)) >> 4) + t[1]);
            st[first + i] = (uint8_t)(pre <= 63 ? 63 - pre : pre - 64);
            mps[first + i] = pre > 63;
        }
    }
}

static void cabd_start(cabd_t *c, br_t *b, int slice_i, int qp) {
    jmo_cabac_init_models(slice_i, qp, c->st, c->mps);
    c->b = b;
    c->range = 510;                                 /* 9.3.1.2 */
    c->ofs = rbits(b, 9);
}
static int cdec(cabd_t *c, int ctx) {               /* DecodeDecision (9.3.3.2.1) */
    uint32_t lps = jmo_lps_range[c->st[ctx]][(c->range >> 6) & 3];
    int bin;
    c->range -= lps;
    if (c->ofs >= c->range) {
        bin = !c->mps[ctx];
        c->ofs -= c->range;
        c->range = lps;
        if (!c->st[ctx]) c->mps[ctx] = !c->mps[ctx];
        c->st[ctx] = jmo_lps_next[c->st[ctx]];
    } else {
        bin = c->mps[ctx];
        if (c->st[ctx] < 62) c->st[ctx]++;
    }
    while (c->range < 256) { c->range <<= 1; c->ofs = (c->ofs << 1) | (uint32_t)rb(c->b); }
    return bin;
}
static int cbypass(cabd_t *c) {
    c->ofs = (c->ofs << 1) | (uint32_t)rb(c->b);
    if (c->ofs >= c->range) { c->ofs -= c->range; return 1; }
    return 0;
}
static int cterm(cabd_t *c) {
    c->range -= 2;
    if (c->ofs >= c->range) return 1;
    while (c->range < 256) { c->range <<= 1; c->ofs = (c->ofs << 1) | (uint32_t)rb(c->b); }
    return 0;
}
static unsigned ceg_bypass(cabd_t *c, int k) {       /* k-th order Exp-Golomb suffix (9.3.2.3) */
    unsigned v = 0;
    while (cbypass(c)) { v += 1u << k; if (++k > 24) return v; }
    while (k--) v += (unsigned)cbypass(c) << k;
    return v;
}

/* Table 9-43: 8x8 frame significant / last ctxIdxInc by scanning position (shared with cabac_enc.c) */
const uint8_t jmo_sig8x8_inc[63] = {0, 1, 2, 3, 4, 5, 5, 4, 4, 3, 3, 4, 4, 4, 5, 5, 4, 4, 4, 4, 3, 3, 6, 7, 7, 7, 8, 9, 10, 9, 8, 7,
                                   7, 6, 11, 12, 13, 11, 6, 7, 8, 9, 14, 10, 9, 8, 6, 11, 12, 13, 11, 6, 9, 14, 10, 9, 11, 12, 13, 11, 14, 10, 12};
const uint8_t jmo_last8x8_inc[63] = {0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2,
                                   3, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7, 8, 8, 8};

/* residual_block_cabac: coef[0..n) scan order; cbfctx < 0: coded_block_flag not coded (8x8) */
static int cabac_block(cabd_t *c, int cat, int n, int cbfctx, int *coef) {
    static const int so[5] = {0, 15, 29, 44, 47}, ao[5] = {0, 10, 20, 30, 39};
    const uint8_t *s8 = jmo_sig8x8_inc, *l8 = jmo_last8x8_inc;
    for (int i = 0; i < n; i++) coef[i] = 0;
    if (cbfctx >= 0 && !cdec(c, cbfctx)) return 0;
    int sbase = cat == 5 ? 402 : 105 + so[cat], lbase = cat == 5 ? 417 : 166 + so[cat], abase = cat == 5 ? 426 : 227 + ao[cat];
    int sig[64] = {0}, lastpos = -1;
    for (int i = 0; i < n - 1 && lastpos < 0; i++) {
        int inc_s = cat == 5 ? s8[i] : cat == 3 ? imin(i, 2) : i, inc_l = cat == 5 ? l8[i] : cat == 3 ? imin(i, 2) : i;
        if (cdec(c, sbase + inc_s)) { sig[i] = 1; if (cdec(c, lbase + inc_l)) lastpos = i; }
    }
    if (lastpos < 0) { lastpos = n - 1; sig[n - 1] = 1; }
    int eq1 = 0, gt1 = 0;
    for (int i = lastpos; i >= 0; i--) {
        if (!sig[i]) continue;
        int v = 0;
        if (cdec(c, abase + (gt1 ? 0 : imin(4, 1 + eq1)))) {
            int ctx = abase + 5 + imin(4 - (cat == 3), gt1);
            v = 1;
            while (v < 14 && cdec(c, ctx)) v++;
            if (v == 14) v += (int)ceg_bypass(c, 0);
        }
        coef[i] = cbypass(c) ? -(v + 1) : v + 1;
        if (v == 0) eq1++; else gt1++;
    }
    return 1;
}

/* mvd_l0 component: UEG3, signed, uCoff 9; bin 0 ctxIdxInc from absMvdComp(A) + absMvdComp(B) */
static int cabac_mvd(cabd_t *c, int comp, int sum) {
    int base = comp ? 47 : 40;
    if (!cdec(c, base + (sum < 3 ? 0 : sum <= 32 ? 1 : 2))) return 0;
    int a = 1;
    while (a < 9 && cdec(c, base + imin(a + 2, 6))) a++;
    if (a == 9) a += (int)ceg_bypass(c, 3);
    return cbypass(c) ? -a : a;
}
/* absMvdComp of the neighbouring partition covering luma (xN, yN) relative to the MB (6.4.11.7) */
static int mvd_abs_nb(const jmo_dec *d, int mx, int my, int xN, int yN, int comp) {
    int tx = xN < 0 ? mx - 1 : mx, ty = yN < 0 ? my - 1 : my;
    if ((tx != mx || ty != my) && !avail_mb(d, tx, ty, mx, my)) return 0;
    int W4 = d->W / 4, i = ((16 * my + yN) >> 2) * W4 + ((16 * mx + xN) >> 2);
    return iabs(d->mvd[2 * i + comp]);
}
static void cabac_part(jmo_dec *d, int mx, int my, int x, int y, int w, int h, mbsyn *s) {
    int p[2], dm[2];
    mvpred(d, mx, my, x, y, w, h, 0, p);
    for (int comp = 0; comp < 2; comp++)
        dm[comp] = cabac_mvd(&d->cab, comp, mvd_abs_nb(d, mx, my, x - 1, y, comp) + mvd_abs_nb(d, mx, my, x, y - 1, comp));
    set_part(d, mx, my, x, y, w, h, p[0] + dm[0], p[1] + dm[1], 0, s->mv16);
    int W4 = d->W / 4;
    for (int yy = y; yy < y + h; yy += 4)
        for (int xx = x; xx < x + w; xx += 4) {
            int i = ((16 * my + yy) >> 2) * W4 + ((16 * mx + xx) >> 2);
            d->mvd[2 * i] = (int16_t)dm[0]; d->mvd[2 * i + 1] = (int16_t)dm[1];
        }
}

/* coded_block_flag condTermFlagN of a luma 4x4 block (x4, y4) of neighbour n (9.3.3.1.1.9) */
static int cbf_luma_nb(const mbinfo *n, int x4, int y4, int cur_intra) {
    if (!n) return cur_intra;
    if (n->mbtype == 3) return 0;
    if (!((n->cbp >> ((y4 >> 1) * 2 + (x4 >> 1))) & 1)) return 0;
    if (n->t8) return 1;                             /* 8x8 block: flag inferred 1 */
    return (n->cbf4 >> (y4 * 4 + x4)) & 1;
}

static int parse_cabac(jmo_dec *d, int mx, int my, int slice_p, mbsyn *s, int *qp) {
    cabd_t *c = &d->cab;
    mbinfo *mi = &d->mi[my * d->mbw + mx];
    const mbinfo *A = avail_mb(d, mx - 1, my, mx, my) ? &d->mi[my * d->mbw + mx - 1] : NULL;
    const mbinfo *B = avail_mb(d, mx, my - 1, mx, my) ? &d->mi[(my - 1) * d->mbw + mx] : NULL;
    if (slice_p && cdec(c, 11 + (A && A->mbtype != 3) + (B && B->mbtype != 3))) {   /* mb_skip_flag */
        skip_motion(d, mx, my, s);
        d->prev_qpd = 0;
        return 0;
    }
    /* mb_type */
    int intra = 1, ptype = 0, i16 = 0, cbp = 0;
    if (slice_p) intra = cdec(c, 14);
    if (intra) {
        int o = slice_p ? 17 : 3;
        int inc = slice_p ? 0 : (A && A->mbtype != 1 && A->mbtype != 4) + (B && B->mbtype != 1 && B->mbtype != 4);
        i16 = cdec(c, o + inc);
        if (i16) {
            if (cterm(c)) FAIL("I_PCM unsupported");
            int luma = cdec(c, slice_p ? 18 : 6), chroma = cdec(c, slice_p ? 19 : 7);
            if (chroma) chroma += cdec(c, slice_p ? 19 : 8);
            int pm = cdec(c, slice_p ? 20 : 9) << 1;
            pm |= cdec(c, slice_p ? 20 : 10);
            s->i16mode = pm;
            cbp = (chroma << 4) | (luma ? 15 : 0);
        }
    } else {
        int b1 = cdec(c, 15), b2 = cdec(c, 16 + b1);
        ptype = b1 ? (b2 ? 1 : 2) : (b2 ? 3 : 0);       /* 0 16x16, 1 16x8, 2 8x16, 3 8x8 */
    }
    int no_sub8x8 = 1;
    if (intra) {
        s->intra_type = i16 ? 1 : 0;
        mi->intra = 1;
        mi->mbtype = i16 ? 2 : 1;
        if (!i16) {
            if (d->t8mode) mi->t8 = cdec(c, 399 + (A && A->t8) + (B && B->t8));
            if (mi->t8) mi->mbtype = 4;
            for (int blk = 0; blk < 16; blk += mi->t8 ? 4 : 1) {
                int x4 = ((blk >> 2) & 1) * 2 + (blk & 1), y4 = (blk >> 3) * 2 + ((blk >> 1) & 1);
                int pm = pred_ipm(d, mx, my, x4, y4, s->ipm), mode = pm;
                if (!cdec(c, 68)) {
                    int rem = cdec(c, 69);
                    rem |= cdec(c, 69) << 1;
                    rem |= cdec(c, 69) << 2;
                    mode = rem < pm ? rem : rem + 1;
                }
                set_ipm(s, x4, y4, mode, mi->t8);
            }
            for (int k = 0; k < 16; k++) mi->ipm[k] = (int8_t)s->ipm[k];
        }
        int ia = A && A->intra && A->cmode, ib = B && B->intra && B->cmode;
        s->cmode = cdec(c, 64 + ia + ib);
        if (s->cmode) { s->cmode += cdec(c, 67); if (s->cmode == 2) s->cmode += cdec(c, 67); }
        mi->cmode = s->cmode;
    } else {
        s->intra_type = -1;
        mi->mbtype = 0;
        if (ptype == 3) {
            int sub[4];                                  /* 0 8x8, 1 8x4, 2 4x8, 3 4x4 */
            for (int i = 0; i < 4; i++) {
                if (cdec(c, 21)) sub[i] = 0;
                else if (!cdec(c, 22)) sub[i] = 1;
                else sub[i] = cdec(c, 23) ? 2 : 3;
                if (sub[i]) no_sub8x8 = 0;
            }
            for (int i = 0; i < 4; i++) {
                int ox = (i & 1) * 8, oy = (i >> 1) * 8;
                int sw = sub[i] <= 1 ? 8 : 4, sh = (sub[i] == 0 || sub[i] == 2) ? 8 : 4;
                for (int y = 0; y < 8; y += sh)
                    for (int x = 0; x < 8; x += sw) cabac_part(d, mx, my, ox + x, oy + y, sw, sh, s);
            }
        } else {
            int np = ptype == 0 ? 1 : 2, w = ptype == 2 ? 8 : 16, h = ptype == 1 ? 8 : 16;
            for (int pi = 0; pi < np; pi++) cabac_part(d, mx, my, ptype == 2 ? 8 * pi : 0, ptype == 1 ? 8 * pi : 0, w, h, s);
        }
    }
    if (!i16) {                                           /* coded_block_pattern */
        for (int b8 = 0; b8 < 4; b8++) {
            int ta = (b8 & 1) ? !((cbp >> (b8 - 1)) & 1) : A ? !((A->cbp >> (b8 + 1)) & 1) : 0;
            int tb = (b8 & 2) ? !((cbp >> (b8 - 2)) & 1) : B ? !((B->cbp >> (b8 + 2)) & 1) : 0;
            cbp |= cdec(c, 73 + ta + 2 * tb) << b8;
        }
        int ca = A ? A->cbp >> 4 : 0, cb = B ? B->cbp >> 4 : 0;
        if (cdec(c, 77 + (ca != 0) + 2 * (cb != 0))) cbp |= (1 + cdec(c, 81 + (ca == 2) + 2 * (cb == 2))) << 4;
        if (!intra && (cbp & 15) && d->t8mode && no_sub8x8) mi->t8 = cdec(c, 399 + (A && A->t8) + (B && B->t8));
    }
    s->cbp = cbp;
    mi->cbp = cbp;
    if (!(cbp > 0 || i16)) { d->prev_qpd = 0; return 0; }
    /* mb_qp_delta: U binarisation of the mapped value, ctxIdx 60..63 */
    int k = 0;
    if (cdec(c, 60 + d->prev_qpd)) { k = 1; while (cdec(c, k == 1 ? 62 : 63)) { if (++k > 104) FAIL("mb_qp_delta"); } }
    int dq = (k & 1) ? (k + 1) / 2 : -(k / 2);
    d->prev_qpd = dq != 0;
    *qp = (*qp + dq + 52 + 2 * d->qpbd) % (52 + d->qpbd) - d->qpbd;
    /* residual */
    int cur_intra = intra, cbpl = cbp & 15, cbpc = cbp >> 4;
    if (i16) {
        int ta = A ? (A->mbtype == 2 ? A->cbf_dc & 1 : 0) : 1, tb = B ? (B->mbtype == 2 ? B->cbf_dc & 1 : 0) : 1;
        mi->cbf_dc |= cabac_block(c, 0, 16, 85 + ta + 2 * tb, s->dc16);
    }
    for (int b8 = 0; b8 < 4; b8++) {
        if (!((cbpl >> b8) & 1)) continue;
        if (mi->t8) {
            cabac_block(c, 5, 64, -1, s->l8[b8]);
            continue;
        }
        for (int i4 = 0; i4 < 4; i4++) {
            int x4 = (b8 & 1) * 2 + (i4 & 1), y4 = (b8 >> 1) * 2 + (i4 >> 1);
            int ta = x4 ? (mi->cbf4 >> (y4 * 4 + x4 - 1)) & 1 : cbf_luma_nb(A, 3, y4, cur_intra);
            int tb = y4 ? (mi->cbf4 >> ((y4 - 1) * 4 + x4)) & 1 : cbf_luma_nb(B, x4, 3, cur_intra);
            int f = i16 ? cabac_block(c, 1, 15, 89 + ta + 2 * tb, s->l4[y4 * 4 + x4] + 1)
                        : cabac_block(c, 2, 16, 93 + ta + 2 * tb, s->l4[y4 * 4 + x4]);
            mi->cbf4 |= f << (y4 * 4 + x4);
        }
    }
    if (cbpc)
        for (int comp = 0; comp < 2; comp++) {
            int ta = !A ? cur_intra : (A->mbtype == 3 || !(A->cbp >> 4)) ? 0 : (A->cbf_dc >> (1 + comp)) & 1;
            int tb = !B ? cur_intra : (B->mbtype == 3 || !(B->cbp >> 4)) ? 0 : (B->cbf_dc >> (1 + comp)) & 1;
            mi->cbf_dc |= cabac_block(c, 3, 4, 97 + ta + 2 * tb, s->cdc[comp]) << (1 + comp);
        }
    if (cbpc == 2)
        for (int comp = 0; comp < 2; comp++)
            for (int k4 = 0; k4 < 4; k4++) {
                int ta = (k4 & 1) ? (mi->cbfc[comp] >> (k4 - 1)) & 1
                         : !A ? cur_intra : (A->mbtype == 3 || (A->cbp >> 4) != 2) ? 0 : (A->cbfc[comp] >> (k4 + 1)) & 1;
                int tb = (k4 & 2) ? (mi->cbfc[comp] >> (k4 - 2)) & 1
                         : !B ? cur_intra : (B->mbtype == 3 || (B->cbp >> 4) != 2) ? 0 : (B->cbfc[comp] >> (k4 + 2)) & 1;
                mi->cbfc[comp] |= cabac_block(c, 4, 15, 101 + ta + 2 * tb, s->cac[comp][k4] + 1) << k4;
            }
    return c->b->err ? -1 : 0;
}

/* prediction + residual reconstruction of a parsed macroblock (8.3, 8.4, 8.5) */
static int recon_mb(jmo_dec *d, int mx, int my, const mbsyn *s, int qp_) {
    mbinfo *mi = &d->mi[my * d->mbw + mx];
    mi->qp = qp_;
    mi->cbp = s->cbp;
    pel pred[256], predu[64], predv[64];
    int intra_type = s->intra_type;
    if (intra_type < 0) inter_pred(d, mx, my, s->mv16, pred, predu, predv);
    else {
        if (predc(d, mx, my, 1, s->cmode, predu) || predc(d, mx, my, 2, s->cmode, predv)) FAIL("chroma pred mode %d unavailable at MB %d,%d", s->cmode, mx, my);
        if (intra_type == 1 && pred16(d, mx, my, s->i16mode, pred)) FAIL("I16 mode %d unavailable at MB %d,%d", s->i16mode, mx, my);
    }
    if (s->skip) mi->cbp = 0;
    /* QPY of the MB is qp_; scaling at QP'Y = QPY + QpBdOffsetY and QP'C = QPC + QpBdOffsetC (8.5.8) */
    const int qpi = iclip(-d->qpbd, 51, qp_ + d->cqp_off), maxv = d->maxv;
    int qpc = (qpi < 0 ? qpi : QPCt[qpi]) + d->qpbd;
    qp_ += d->qpbd;
    int cbpc = s->cbp >> 4;
    int32_t dcY[16] = {0};
    pel *RY = d->cur[0];
    int W = d->W;
    if (intra_type == 1) {
        int32_t m[16], t2[16];
        for (int k = 0; k < 16; k++) m[zz[k]] = s->dc16[k];
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
                dcY[4 * y + x] = qp_ >= 36 ? f[y] * ls * (1 << (qp_ / 6 - 6)) : (f[y] * ls + (1 << (5 - qp_ / 6))) >> (6 - qp_ / 6);
            }
        }
    }
    for (int b8 = 0; b8 < 4 && mi->t8; b8++) {       /* 8x8 transform */
        int any = 0;
        for (int k = 0; k < 64; k++) any |= s->l8[b8][k] != 0;
        int bx = 8 * (b8 & 1), by = 8 * (b8 >> 1);
        if (any) mi->nzblk |= 0x33 << ((by >> 2) * 4 + (bx >> 2));
        pel *dst = RY + (16 * my + by) * W + 16 * mx + bx;
        if (intra_type == 0) {
            pel p64[64];
            if (pred8x8(d, mx, my, b8, s->ipm[(by >> 2) * 4 + (bx >> 2)], p64)) FAIL("I8 mode unavailable at MB %d,%d", mx, my);
            recon8x8(s->l8[b8], qp_, p64, 8, dst, W, maxv);
        } else recon8x8(s->l8[b8], qp_, pred + by * 16 + bx, 16, dst, W, maxv);
    }
    for (int blk = 0; blk < 16 && !mi->t8; blk++) {
        int b8 = blk >> 2;
        int x4 = (b8 & 1) * 2 + (blk & 1), y4 = (b8 >> 1) * 2 + ((blk >> 1) & 1);
        const int *c = s->l4[y4 * 4 + x4];
        int any = 0;
        for (int k = 0; k < 16; k++) any |= c[k] != 0;
        if (any) mi->nzblk |= 1 << (y4 * 4 + x4);
        int32_t m[16];
        for (int k = 0; k < 16; k++) m[zz[k]] = c[k];
        scale4x4(m, qp_, intra_type == 1);
        if (intra_type == 1) m[0] = dcY[y4 * 4 + x4];
        pel *dst = RY + (16 * my + 4 * y4) * W + 16 * mx + 4 * x4;
        if (intra_type == 0) {
            pel p4[16];
            int ok;
            pred4x4(d, mx, my, 4 * x4, 4 * y4, blk, s->ipm[y4 * 4 + x4], p4, &ok);
            if (!ok) FAIL("I4 mode %d unavailable at MB %d,%d blk %d", s->ipm[y4 * 4 + x4], mx, my, blk);
            recon4x4(m, p4, 4, dst, W, maxv);
        } else recon4x4(m, pred + 4 * y4 * 16 + 4 * x4, 16, dst, W, maxv);
    }
    int dcc[2][4] = {{0}};
    if (cbpc)
        for (int comp = 0; comp < 2; comp++) {
            const int *c = s->cdc[comp];
            int f[4] = {c[0] + c[1] + c[2] + c[3], c[0] - c[1] + c[2] - c[3], c[0] + c[1] - c[2] - c[3], c[0] - c[1] - c[2] + c[3]};
            for (int k = 0; k < 4; k++) dcc[comp][k] = (f[k] * lscale(qpc % 6, 0) * (1 << (qpc / 6))) >> 5;
        }
    for (int comp = 0; comp < 2; comp++) {
        pel *R = d->cur[1 + comp];
        int Wc = d->W / 2;
        for (int k = 0; k < 4; k++) {
            int32_t m[16];
            for (int q = 0; q < 16; q++) m[zz[q]] = s->cac[comp][k][q];
            scale4x4(m, qpc, 1);
            m[0] = dcc[comp][k];
            int xo = (k & 1) * 4, yo = (k >> 1) * 4;
            recon4x4(m, (comp ? predv : predu) + yo * 8 + xo, 8, R + (8 * my + yo) * Wc + 8 * mx + xo, Wc, maxv);
        }
    }
    return 0;
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
/* alpha, beta, tC0 times 1 << (BitDepth - 8) (8-460, 8-461, 8-470); Clip1 to maxv */
static void edge_filter(pel *s, int step, int bS, int qpav, int chroma, int offA, int offB, int bd) {
    int iA = iclip(0, 51, qpav + offA), iB = iclip(0, 51, qpav + offB), sc = 1 << (bd - 8), maxv = (1 << bd) - 1;
    int a = Alpha[iA] * sc, bt = Beta[iB] * sc;
    int p0 = s[-step], p1 = s[-2 * step], q0 = s[0], q1 = s[step];
    if (!(bS && iabs(p0 - q0) < a && iabs(p1 - p0) < bt && iabs(q1 - q0) < bt)) return;
    if (bS < 4) {
        int tc0 = Tc0[iA][bS - 1] * sc, tc;
        if (chroma) tc = tc0 + 1;
        else {
            int p2 = s[-3 * step], q2 = s[2 * step];
            int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
            tc = tc0 + (ap < bt) + (aq < bt);
            if (ap < bt) s[-2 * step] = (pel)(p1 + iclip(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - 2 * p1) >> 1));
            if (aq < bt) s[step] = (pel)(q1 + iclip(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - 2 * q1) >> 1));
        }
        int dl = iclip(-tc, tc, ((q0 - p0) * 4 + (p1 - q1) + 4) >> 3);
        s[-step] = (pel)iclip(0, maxv, p0 + dl);
        s[0] = (pel)iclip(0, maxv, q0 - dl);
    } else if (chroma) {
        s[-step] = (pel)((2 * p1 + p0 + q1 + 2) >> 2);
        s[0] = (pel)((2 * q1 + q0 + p1 + 2) >> 2);
    } else {
        int p2 = s[-3 * step], q2 = s[2 * step], p3 = s[-4 * step], q3 = s[3 * step];
        int ap = iabs(p2 - p0), aq = iabs(q2 - q0), sm = iabs(p0 - q0) < ((a >> 2) + 2);
        if (ap < bt && sm) {
            s[-step] = (pel)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
            s[-2 * step] = (pel)((p2 + p1 + p0 + q0 + 2) >> 2);
            s[-3 * step] = (pel)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
        } else s[-step] = (pel)((2 * p1 + p0 + q1 + 2) >> 2);
        if (aq < bt && sm) {
            s[0] = (pel)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
            s[step] = (pel)((p0 + q0 + q1 + q2 + 2) >> 2);
            s[2 * step] = (pel)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
        } else s[0] = (pel)((2 * q1 + q0 + p1 + 2) >> 2);
    }
}
/* QPc of a macroblock's QPY (8.5.8, qPI clipped to [-QpBdOffsetC, 51]) for the chroma filter */
static int qpc_of(const jmo_dec *d, int qpy) {
    int qpi = iclip(-d->qpbd, 51, qpy + d->cqp_off);
    return qpi < 0 ? qpi : QPCt[qpi];
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
                    int qcav = (qpc_of(d, qp_) + qpc_of(d, qq) + 1) >> 1;
                    for (int k = 0; k < 16; k++) {
                        int xq = vert ? 16 * mx + e : 16 * mx + k, yq = vert ? 16 * my + k : 16 * my + e;
                        int bS = bs_of(d, vert ? xq - 1 : xq, vert ? yq : yq - 1, xq, yq, e == 0);
                        edge_filter(d->cur[0] + yq * W + xq, vert ? 1 : W, bS, qav, 0, d->offA, d->offB, d->bd);
                        if ((e & 7) == 0 && (k & 1) == 0) {
                            int cx = vert ? 8 * mx + e / 2 : 8 * mx + k / 2, cy = vert ? 8 * my + k / 2 : 8 * my + e / 2;
                            for (int c = 1; c <= 2; c++) {
                                edge_filter(d->cur[c] + cy * Wc + cx, vert ? 1 : Wc, bS, qcav, 1, d->offA, d->offB, d->bd);
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
    if (d->cabac && st == 0 && rue(b) != 0) FAIL("cabac_init_idc other than 0 unsupported");
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
    mbsyn syn;
    if (d->cabac) {                            /* slice_data with CABAC (7.3.4) */
        while (b->pos & 7) if (!rb(b)) FAIL("cabac_alignment_one_bit");
        cabd_start(&d->cab, b, st == 2, qp);
        d->prev_qpd = 0;
        while (a < nmb) {
            int mx = a % d->mbw, my = a / d->mbw;
            mb_begin(d, mx, my, &syn);
            if (parse_cabac(d, mx, my, st == 0, &syn, &qp) || recon_mb(d, mx, my, &syn, qp)) return -1;
            a++;
            if (b->err) FAIL("CABAC slice data overrun at MB %d", a);
            if (cterm(&d->cab)) break;             /* end_of_slice_flag */
        }
    }
    while (!d->cabac && more && a < nmb) {
        if (st == 0) {
            int run = rue(b);
            if (b->err) FAIL("skip run");
            for (int i = 0; i < run && a < nmb; i++, a++) {
                mb_begin(d, a % d->mbw, a / d->mbw, &syn);
                skip_motion(d, a % d->mbw, a / d->mbw, &syn);
                if (recon_mb(d, a % d->mbw, a / d->mbw, &syn, qp)) return -1;
            }
            if (run > 0) more = more_rbsp_data(b);
        }
        if (more && a < nmb) {
            int t = rue(b);
            if (b->err) FAIL("mb_type at MB %d", a);
            int mx = a % d->mbw, my = a / d->mbw;
            mb_begin(d, mx, my, &syn);
            if (parse_cavlc(d, b, mx, my, st == 0, t, &syn, &qp) || recon_mb(d, mx, my, &syn, qp)) return -1;
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
                const int ps = d->bd > 8 ? 2 : 1;          /* output: bytes, or 16-bit LE samples (High 10) */
                long fs = (long)cw * ch * 3 / 2 * ps;
                if ((nframes + 1) * fs > out_cap) { snprintf(d->err, sizeof d->err, "output buffer too small"); r = -1; }
                else {
                    uint8_t *o = out + nframes * fs;
                    long k = 0;
                    for (int c = 0; c < 3; c++) {
                        const int pw = c ? cw / 2 : cw, ph = c ? ch / 2 : ch, st = c ? d->W / 2 : d->W;
                        const int ox = c ? d->crop_l : 2 * d->crop_l, oy = c ? d->crop_t : 2 * d->crop_t;
                        for (int y = 0; y < ph; y++)
                            for (int x = 0; x < pw; x++, k++) {
                                const pel v = d->cur[c][(long)(y + oy) * st + ox + x];
                                if (ps == 1) o[k] = (uint8_t)v;
                                else { o[2 * k] = (uint8_t)v; o[2 * k + 1] = (uint8_t)(v >> 8); }
                            }
                    }
                    nframes++;
                    *width = cw; *height = ch;
                    for (int c = 0; c < 3; c++) { pel *t = d->ref[c]; d->ref[c] = d->cur[c]; d->cur[c] = t; }
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
